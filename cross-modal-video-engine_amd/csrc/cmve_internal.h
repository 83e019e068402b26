// Internal helpers shared by the libcmve.so translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <string>
#include "../../include/cmve.h"

struct cmve_handle {
  int device;
  hipStream_t stream;
};

namespace cmve {

void set_error(const char* fmt, ...);
int check_launch(const char* what);

#define CMVE_REQUIRE(cond, ...)            \
  do {                                     \
    if (!(cond)) {                         \
      ::cmve::set_error(__VA_ARGS__);      \
      return CMVE_E_INVALID;               \
    }                                      \
  } while (0)

#define CMVE_HIP(call)                                                              \
  do {                                                                              \
    hipError_t e_ = (call);                                                         \
    if (e_ != hipSuccess) {                                                         \
      ::cmve::set_error("%s failed: %s", #call, hipGetErrorString(e_));            \
      return CMVE_E_HIP;                                                            \
    }                                                                               \
  } while (0)

constexpr int WAVE = 64;

// ---- bf16 <-> f32 (round to nearest even; NaN stays NaN) ----
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }

// ---- wave reductions (xor butterfly: every lane ends with bit-identical sums) ----
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T> __device__ __forceinline__ double ld64(const T* p) { return (double)(*p); }

// Exact-ish fp64 dot of two raw rows: lane-strided fma chains then a butterfly.
// The SAME routine serves the GT scores and the fix-up, so a pair scored in both
// places gets bit-identical values.
template <typename TA, typename TB>
__device__ __forceinline__ double wave_dot64(const TA* __restrict__ a, const TB* __restrict__ b,
                                             int64_t d, int lane) {
  double acc = 0.0;
  for (int64_t k = lane; k < d; k += WAVE) acc = fma(ld64(a + k), ld64(b + k), acc);
  return wave_sum(acc);
}

// fp64 -> fp32 with directed rounding
__device__ __forceinline__ float f32_round_up(double x) {
  float f = (float)x;
  if ((double)f < x) f = nextafterf(f, INFINITY);
  return f;
}
__device__ __forceinline__ float f32_round_down(double x) {
  float f = (float)x;
  if ((double)f > x) f = nextafterf(f, -INFINITY);
  return f;
}

// Rigorous bound on |score_mfma(i,j) - cos_exact(i,j)| for row errors ea, eb:
//   representation:  ea + (1 + ea) * eb          (Cauchy-Schwarz on x_hat - x_tilde)
//   accumulation:    gamma_n * (1 + ea) * (1 + eb)
// n counts roundings as if every product and the C operand of each 32-deep
// v_mfma_f32_16x16x32 were added with its own rounding (33 per 32 products), at
// u = 2^-23 (2x RNE: covers the truncating alignment the MFMA probe shows -- it drops
// product bits below ~2^-24 of the largest term, tests/test_gpu_numerics.py).
__host__ __device__ __forceinline__ double score_error_bound(double ea, double eb, int64_t d_pad, int mode) {
  const double n = (double)d_pad * (33.0 / 32.0) * (mode == CMVE_SIM_BF16X3 ? 3.0 : 1.0);
  const double u = 1.0 / 8388608.0;  // 2^-23
  const double gamma = n * u / (1.0 - n * u);
  return ea + (1.0 + ea) * eb + gamma * (1.0 + ea) * (1.0 + eb) + 1e-12;
}

// per-row error plane and err_max slot of a sim mode (err_max = {hi, hilo, h16})
inline const float* mode_err(const cmve_rows_t* r, int mode) {
  return mode == CMVE_SIM_BF16 ? r->err_hi : (mode == CMVE_SIM_BF16X3 ? r->err_hilo : r->err_h16);
}
__host__ __device__ __forceinline__ int mode_slot(int mode) { return mode; }

}  // namespace cmve
