// Internal helpers shared by the libcmve.so translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <string>
#include <algorithm>
#include <type_traits>
#include "../../include/cmve.h"

struct cmve_handle {
  int device;
  hipStream_t stream;
  // auxiliary stream + events for cmve_rank_count_overlap (created on first use)
  hipStream_t aux = nullptr;
  hipEvent_t ev[CMVE_MAX_CHUNKS + 2] = {};
  hipEvent_t tev[2 * CMVE_MAX_CHUNKS] = {};  // timing: around each chunk's MFMA pass
  int last_chunks = 0;
  // grow-only device scratch (split-K partials of cmve_gemm_f32); grown outside the hot loop
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
};

namespace cmve {

void set_error(const char* fmt, ...);
int check_launch(const char* what);
// make h->scratch at least `bytes` (synchronises the stream and reallocates only when it grows)
int ensure_scratch(cmve_handle* h, size_t bytes);

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
//
// fp32 x fp32 rows with d % 4 == 0 and 16-B aligned starts (the bench / evaluation layout): lane
// L owns elements 4L + 256m + c, c = 0..3, accumulated in (m, c) order from float4 loads, four
// 256-element strides per trip so eight 16-B loads are in flight (the fix-up re-scores ~1e6
// random pairs: latency, not arithmetic, bounds it).  The order is a function of the pair alone
// and symmetric in (a, b), so every caller still gets the same bits for the same pair.
template <typename TA, typename TB>
__device__ __forceinline__ double wave_dot64(const TA* __restrict__ a, const TB* __restrict__ b,
                                             int64_t d, int lane) {
  double acc = 0.0;
  if constexpr (std::is_same<TA, float>::value && std::is_same<TB, float>::value) {
    if ((d & 3) == 0 && ((((uintptr_t)a) | ((uintptr_t)b)) & 15) == 0) {
      auto fma4 = [&](const float4& x, const float4& y) {
        acc = fma((double)x.x, (double)y.x, acc);
        acc = fma((double)x.y, (double)y.y, acc);
        acc = fma((double)x.z, (double)y.z, acc);
        acc = fma((double)x.w, (double)y.w, acc);
      };
      int64_t k = (int64_t)lane * 4;
      for (; k + 768 < d; k += 1024) {
        const float4 a0 = *(const float4*)(a + k), a1 = *(const float4*)(a + k + 256);
        const float4 a2 = *(const float4*)(a + k + 512), a3 = *(const float4*)(a + k + 768);
        const float4 b0 = *(const float4*)(b + k), b1 = *(const float4*)(b + k + 256);
        const float4 b2 = *(const float4*)(b + k + 512), b3 = *(const float4*)(b + k + 768);
        fma4(a0, b0);
        fma4(a1, b1);
        fma4(a2, b2);
        fma4(a3, b3);
      }
      for (; k < d; k += 256) fma4(*(const float4*)(a + k), *(const float4*)(b + k));
      return wave_sum(acc);
    }
  }
  for (int64_t k = lane; k < d; k += WAVE) acc = fma(ld64(a + k), ld64(b + k), acc);
  return wave_sum(acc);
}

// order-preserving uint32 key of an fp32 score (larger score -> larger key); NaN -> 0 (ranks
// last, as np.argsort puts NaN errors last)
__device__ __forceinline__ uint32_t topk_key(float f) {
  const uint32_t u = __float_as_uint(f);
  if (f != f) return 0u;
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float topk_key_inv(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
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

// Undecided-pair buffer layout (cand, cap uint64 entries), derived from the gallery set alone:
//   cand[0, nb)                       per-bucket pair counters
//   cand[nb + b*cap_b, +cap_b)        bucket b: pairs whose gallery row j has j >> 8 == b
// Bucketing by 256 gallery rows lets the fix-up re-score a bucket's pairs while its 1 MiB of raw
// gallery rows sits in one XCD's L2 (each gallery row has ~10 pairs): the gallery side is read from
// HBM once instead of once per pair.
constexpr int CAND_BUCKET_SHIFT = 8;
struct CandLayout {
  int64_t nb, cap_b;
};
inline CandLayout cand_layout(int64_t g_n_pad, int64_t cap) {
  CandLayout l;
  l.nb = std::max<int64_t>(1, (g_n_pad + (1 << CAND_BUCKET_SHIFT) - 1) >> CAND_BUCKET_SHIFT);
  l.cap_b = cap > l.nb ? (cap - l.nb) / l.nb : 0;
  return l;
}
constexpr int64_t FIXUP_MAX_BUCKETS_PER_XCD = 4096;  // LDS prefix of the XCD-ordered fix-up

// per-row error plane and err_max slot of a sim mode (err_max = {hi, hilo, h16})
inline const float* mode_err(const cmve_rows_t* r, int mode) {
  return mode == CMVE_SIM_BF16 ? r->err_hi : (mode == CMVE_SIM_BF16X3 ? r->err_hilo : r->err_h16);
}
__host__ __device__ __forceinline__ int mode_slot(int mode) { return mode; }

}  // namespace cmve
