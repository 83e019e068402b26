// MFMA numerics probe: pins the accumulation model the rank epilogue's error bound relies on.
//
// The bound (cmve_internal.h, score_error_bound) charges the fp32 accumulation of one
// similarity score as ROUNDINGS_PER_MFMA roundings per v_mfma_f32_16x16x32_{bf16,f16}.
// This kernel feeds crafted operands whose result differs between accumulation models
// (per-product fma chain vs exact sum + one rounding per instruction, RNE vs truncation)
// and reports what the hardware did; tests/test_gpu_numerics.py asserts the model.
#include "cmve_internal.h"

namespace cmve {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

// One wave.  A[row][k] / B[k][col] for lane l: row/col = l & 15, k = 8 * (l >> 4) + e.
// Case c puts products into column 0 / row 0 only; everything else is zero.
//   out[c] = D[0][0] as raw fp32 bits
__device__ float probe_case(int c, int lane, bool f16) {
  float a[8], b[8];
  for (int e = 0; e < 8; ++e) a[e] = b[e] = 0.f;
  const int row = lane & 15, kbase = 8 * (lane >> 4);
  float cin = 0.f;
  for (int e = 0; e < 8; ++e) {
    const int k = kbase + e;
    float av = 0.f, bv = 0.f;
    switch (c) {
      case 0:  // 1 + 16 * 2^-25 : chain-RNE -> 1 ; exact-then-round -> 1 + 2^-21
        if (k == 0) av = bv = 1.f;
        else if (k <= 16) { av = 0x1p-12f; bv = 0x1p-13f; }
        break;
      case 1:  // 1 + 2 * 2^-24 : chain-RNE (ties to even) -> 1 ; exact -> 1 + 2^-23
        if (k == 0) av = bv = 1.f;
        else if (k <= 2) { av = 0x1p-12f; bv = 0x1p-12f; }
        break;
      case 2:  // 1 + 3 * 2^-25 = 1 + 0.75 ulp : RNE -> 1 + 2^-23 ; truncation -> 1
        if (k == 0) av = bv = 1.f;
        else if (k <= 3) { av = 0x1p-12f; bv = 0x1p-13f; }
        break;
      case 3:  // C = 1, products 3 * 2^-25 (accumulator-side rounding): RNE -> 1 + 2^-23
        if (k >= 1 && k <= 3) { av = 0x1p-12f; bv = 0x1p-13f; }
        break;
      case 4:  // cancellation: 1 - 1 + 2^-30 (k = 0, 31, 5): exact 2^-30
        if (k == 0) av = bv = 1.f;
        else if (k == 31) { av = 1.f; bv = -1.f; }
        else if (k == 5) { av = 0x1p-15f; bv = 0x1p-15f; }
        break;
    }
    if (row == 0) a[e] = av;
    if (row == 0) b[e] = bv;
  }
  if (c == 3) cin = 1.f;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  if (lane >> 4 == 0) acc[0] = cin;  // D[row 0][col 0] is lane 0, reg 0
  if (f16) {
    f16x8_t fa, fb;
    for (int e = 0; e < 8; ++e) {
      fa[e] = (_Float16)a[e];
      fb[e] = (_Float16)b[e];
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa, fb, acc, 0, 0, 0);
  } else {
    bf16x8_t fa, fb;
    for (int e = 0; e < 8; ++e) {
      fa[e] = (__bf16)a[e];
      fb[e] = (__bf16)b[e];
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc, 0, 0, 0);
  }
  return acc[0];
}

__global__ void mfma_probe_kernel(float* out) {
  const int lane = threadIdx.x;
  for (int f = 0; f < 2; ++f)
    for (int c = 0; c < 5; ++c) {
      const float v = probe_case(c, lane, f == 1);
      if (lane == 0) out[f * 5 + c] = v;
    }
}

}  // namespace cmve

extern "C" int cmve_mfma_probe(cmve_handle_t h, float* out10) {
  CMVE_REQUIRE(h && out10, "cmve_mfma_probe: NULL argument");
  hipLaunchKernelGGL(cmve::mfma_probe_kernel, dim3(1), dim3(64), 0, h->stream, out10);
  return cmve::check_launch("mfma_probe_kernel");
}
