// Internal helpers shared by the libcmve.so translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
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
  // timing events of cmve_eval_ranks (a ring of CMVE_EVAL_TIMING_SLOTS x 4, created on first use)
  hipEvent_t eval_ev[CMVE_EVAL_TIMING_SLOTS][4] = {};
  // kernel-exact timing of the same evaluations: start / stop of each of the four launches
  hipEvent_t eval_kev[CMVE_EVAL_TIMING_SLOTS][8] = {};
  bool eval_no_fix[CMVE_EVAL_TIMING_SLOTS] = {};  // the slot's evaluation had no fix-up launch (re-scored in the GEMM)
  bool eval_chained[CMVE_EVAL_TIMING_SLOTS] = {};  // the slot's batch ran chained (its finish in the next run's launch)
  // grow-only device scratch (split-K partials of cmve_gemm_f32); grown outside the hot loop
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  // RCCL communicator of cmve_dist_init (dist.hip), nullptr without one
  void* comm = nullptr;
  int nranks = 1, rank = 0;
};

namespace cmve {

void set_error(const char* fmt, ...);
int check_launch(const char* what);
// make h->scratch at least `bytes` (synchronises the stream and reallocates only when it grows)
int ensure_scratch(cmve_handle* h, size_t bytes);
// destroy the handle's RCCL communicator, if any (dist.hip)
void dist_release(cmve_handle* h);
// k-way merge of sorted top-k runs (merge.hip): entry (q, run l, pos p) at q * q_stride + l * l_stride + p
int merge_topk_launch(hipStream_t s, const int64_t* ids, const double* scores, int64_t n_q, int lists, int k_in,
                      int64_t q_stride, int64_t l_stride, int k_out, int64_t* out_ids, double* out_scores);
// Kernel-exact launch timing: when armed, the next launch made through cmve::launch records its own start
// and stop on these events (hipExtLaunchKernelGGL: the dispatch's timestamps, the duration rocprofv3
// reports -- events recorded around a launch also count its dispatch gap)
struct LaunchEv {
  hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local LaunchEv g_launch_ev;
template <typename F, typename... Args>
inline void launch(F kernel, dim3 grid, dim3 block, uint32_t shmem, hipStream_t s, Args... args) {
  if (g_launch_ev.start) {
    const LaunchEv e = g_launch_ev;
    g_launch_ev = LaunchEv{};
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, e.start, e.stop, 0u, args...);
  } else {
    hipLaunchKernelGGL(kernel, grid, block, shmem, s, args...);
  }
}
// compute units of the current device (queried once per device; thread-safe)
int device_cus();

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

// ---- global-address-space accesses ----
// A pointer the kernel READ from memory (a batch's argument table, cmve_eval_batch_*) has no known address space,
// so plain loads / stores / atomics through it compile to flat_* instructions, whose waits also cover the LDS
// traffic (every lgkmcnt wait of an epilogue or a ring barrier then waits for them too).  These helpers access
// device (global) memory through an address_space(1) view of the pointer: global_* instructions on every path.
#define CMVE_GP(T) __attribute__((address_space(1))) T*
template <typename T> __device__ __forceinline__ T gld(const T* p) { return *(const CMVE_GP(T))p; }
template <typename T, typename U> __device__ __forceinline__ void gst(T* p, U v) { *(CMVE_GP(T))p = (T)v; }
template <typename T> __device__ __forceinline__ T gadd(T* p, T v) {
  return __hip_atomic_fetch_add((CMVE_GP(T))p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T> __device__ __forceinline__ T gmax(T* p, T v) {
  return __hip_atomic_fetch_max((CMVE_GP(T))p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T> __device__ __forceinline__ double ld64(const T* p) { return (double)gld(p); }

typedef float cmve_f32x4 __attribute__((ext_vector_type(4)));
typedef double cmve_f64x2 __attribute__((ext_vector_type(2)));

// four consecutive elements of a raw row as doubles (16-B aligned: one float4 or two double2 loads)
__device__ __forceinline__ void load4d(const float* p, double (&v)[4]) {
  const cmve_f32x4 x = gld((const cmve_f32x4*)p);
  v[0] = x.x;
  v[1] = x.y;
  v[2] = x.z;
  v[3] = x.w;
}
__device__ __forceinline__ void load4d(const double* p, double (&v)[4]) {
  const cmve_f64x2 x = gld((const cmve_f64x2*)p), y = gld((const cmve_f64x2*)(p + 2));
  v[0] = x.x;
  v[1] = x.y;
  v[2] = y.x;
  v[3] = y.y;
}
// rows whose elements 4L + 256m + c a lane may read in 16-B pieces
template <typename T>
__host__ __device__ __forceinline__ bool rows_vec4(const T* p, int64_t d, int64_t ld) {
  return (d & 3) == 0 && ((ld * (int64_t)sizeof(T)) & 15) == 0 && (((uintptr_t)p) & 15) == 0;
}

// Exact-ish fp64 dot of two raw rows: per-lane fma chains then a butterfly.  The SAME routine
// serves the GT scores, the fix-up and the top-k re-score, so a pair scored in two places gets
// bit-identical values.
//
// Rows with d % 4 == 0 and 16-B aligned starts (the bench / evaluation layout, fp32 or fp64): lane
// L owns elements 4L + 256m + c, c = 0..3, accumulated in (m, c) order, four 256-element strides per
// trip so eight 16-B (fp32) or sixteen 16-B (fp64) loads are in flight (the fix-up re-scores random
// pairs: latency, not arithmetic, bounds it).  The order is a function of the pair alone (not of
// the element types) and symmetric in (a, b), so every caller gets the same bits for the same pair.
// LIGHT: the same chain with half the loads in flight (two 256-element strides at a time): the same bits at half the
// registers, for kernels whose register budget the rare fp64 re-score must not set (the chained prep + finish)
template <typename TA, typename TB, bool LIGHT = false>
__device__ __forceinline__ double wave_dot64(const TA* __restrict__ a, const TB* __restrict__ b,
                                             int64_t d, int lane) {
  double acc = 0.0;
  if ((d & 3) == 0 && ((((uintptr_t)a) | ((uintptr_t)b)) & 15) == 0) {
    auto fma4 = [&](const double (&x)[4], const double (&y)[4]) {
#pragma unroll
      for (int c = 0; c < 4; ++c) acc = fma(x[c], y[c], acc);
    };
    int64_t k = (int64_t)lane * 4;
    for (; k + 768 < d; k += 1024) {
      if constexpr (LIGHT) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          double a0[4], a1[4], b0[4], b1[4];
          load4d(a + k + 512 * h, a0);
          load4d(a + k + 512 * h + 256, a1);
          load4d(b + k + 512 * h, b0);
          load4d(b + k + 512 * h + 256, b1);
          fma4(a0, b0);
          fma4(a1, b1);
          __builtin_amdgcn_sched_barrier(0);  // (the next half's loads stay below this half's fmas)
        }
        continue;
      }
      double a0[4], a1[4], a2[4], a3[4], b0[4], b1[4], b2[4], b3[4];
      load4d(a + k, a0);
      load4d(a + k + 256, a1);
      load4d(a + k + 512, a2);
      load4d(a + k + 768, a3);
      load4d(b + k, b0);
      load4d(b + k + 256, b1);
      load4d(b + k + 512, b2);
      load4d(b + k + 768, b3);
      fma4(a0, b0);
      fma4(a1, b1);
      fma4(a2, b2);
      fma4(a3, b3);
    }
    {
      // the last (at most three) 256-element strides with every load in flight before the fmas, which keep the
      // stride order (the same bits): a 640-element row (C4) is one round trip instead of three
      double x[3][4], y[3][4];
#pragma unroll
      for (int m = 0; m < 3; ++m)
        if (k + 256 * m < d) {
          load4d(a + k + 256 * m, x[m]);
          load4d(b + k + 256 * m, y[m]);
        }
#pragma unroll
      for (int m = 0; m < 3; ++m)
        if (k + 256 * m < d) fma4(x[m], y[m]);
    }
    return wave_sum(acc);
  }
  for (int64_t k = lane; k < d; k += WAVE) acc = fma(ld64(a + k), ld64(b + k), acc);
  return wave_sum(acc);
}

// wave_dot64 of two pairs at once: every load of both pairs in flight before either fma chain, each
// chain in wave_dot64's own order (the same bits as two wave_dot64 calls); unaligned pairs take those calls
template <typename TA, typename TB>
__device__ __forceinline__ void wave_dot64_x2(const TA* __restrict__ a, const TB* __restrict__ b,
                                              const TA* __restrict__ a2, const TB* __restrict__ b2, int64_t d,
                                              int lane, double& s1, double& s2) {
  if ((d & 3) == 0 && ((((uintptr_t)a) | ((uintptr_t)b) | ((uintptr_t)a2) | ((uintptr_t)b2)) & 15) == 0) {
    double acc = 0.0, acc2 = 0.0;
    auto fma4 = [](double& s, const double (&x)[4], const double (&y)[4]) {
#pragma unroll
      for (int c = 0; c < 4; ++c) s = fma(x[c], y[c], s);
    };
    int64_t k = (int64_t)lane * 4;
    for (; k + 768 < d; k += 1024) {
      double x[4][4], y[4][4], x2[4][4], y2[4][4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        load4d(a + k + 256 * m, x[m]);
        load4d(b + k + 256 * m, y[m]);
        load4d(a2 + k + 256 * m, x2[m]);
        load4d(b2 + k + 256 * m, y2[m]);
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        fma4(acc, x[m], y[m]);
        fma4(acc2, x2[m], y2[m]);
      }
    }
    for (; k < d; k += 256) {
      double x[4], y[4], x2[4], y2[4];
      load4d(a + k, x);
      load4d(b + k, y);
      load4d(a2 + k, x2);
      load4d(b2 + k, y2);
      fma4(acc, x, y);
      fma4(acc2, x2, y2);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {  // wave_sum of both, interleaved
      acc += __shfl_xor(acc, o, 64);
      acc2 += __shfl_xor(acc2, o, 64);
    }
    s1 = acc;
    s2 = acc2;
    return;
  }
  s1 = wave_dot64(a, b, d, lane);
  s2 = wave_dot64(a2, b2, d, lane);
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

// ---- K1 row packing (shared by pack_rows_kernel and the K14 evaluation kernel, so a row packs to the
// same bits on either path) ----
// sum of squares of one raw row in fp64: VEC (fp32, d % 4 == 0, 16-B aligned) float4 runs per lane
template <typename T>
__device__ __forceinline__ double row_sumsq(const T* __restrict__ x, int64_t d, bool vec, int lane) {
  double ss = 0.0;
  if (vec) {  // rows_vec4: elements 4L + 256m + c (fp32 or fp64 alike)
    for (int64_t k = (int64_t)lane * 4; k < d; k += 256) {
      double v[4];
      load4d(x + k, v);
#pragma unroll
      for (int c = 0; c < 4; ++c) ss = fma(v[c], v[c], ss);
    }
    return wave_sum(ss);
  }
  for (int64_t k = lane; k < d; k += WAVE) {
    const double v = (double)x[k];
    ss = fma(v, v, ss);
  }
  return wave_sum(ss);
}
// 1/||x||: eps == 0 is LINAS l2norm (no epsilon: a zero row gives inf, hence NaN elements), eps > 0
// F.normalize; CMVE_PACK_RAW operands are not normalised
__device__ __forceinline__ double row_inv_norm(double ss, double eps, int flags) {
  const double nrm = sqrt(ss);
  return (flags & CMVE_PACK_RAW) ? 1.0 : (eps > 0.0 ? 1.0 / fmax(nrm, eps) : 1.0 / nrm);
}

// one element of a normalised row -> bf16 hi / bf16 lo / fp16 planes, with the squared residuals
// of each representation accumulated in fp64 (the bounds are computed from the values STORED,
// so the f16 conversion need not be correctly rounded from fp64: it goes through fp32, which the
// hardware converts directly -- gfx950 has no fp64 -> fp16 instruction)
struct PackAcc {
  double e1 = 0.0, e2 = 0.0, e3 = 0.0;
  float e4 = 0.f;  // the bf16 residual plane's squared residuals (lo16_elem), summed in fp32
};

// block id -> its XCD's contiguous share of [0, total): the dispatcher deals blocks to the 8 XCDs round robin, so
// XCD x (= bid & 7) walks its own contiguous range in dispatch order and neighbouring work items share its L2
__device__ __forceinline__ int xcd_linear(int bid, int total) {
  const int xcd = bid & 7, local = bid >> 3;
  const int q = total >> 3, r = total & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

// ---- the bf16 residual plane of the fp16 rank operand (K14 level-2 re-score) ----
// An element x (fp64, normalised) is packed as xf = fp32(x), h = fp16(xf); d2 = xf - h is exact in fp32 and
// lo = bf16(d2) (RNE) keeps its top 8 bits: x2 = h + lo with |x - x2| <= |x - xf| + |d2 - lo|, where
// d2 - lo is exact in fp32 and |x - xf| <= 2^-24 |x|.  The bound over a row is therefore
//   ||x - x2|| <= sqrt(sum (d2 - lo)^2) + 2^-24 ||x||     (the fp32 sum's relative error <= 1024 * 2^-24 < 1e-4)
// lo16_elem returns lo's bits and the fp32 residual d2 - lo.
__device__ __forceinline__ uint16_t lo16_elem(float xf, _Float16 h, float& res) {
  const float d2 = xf - (float)h;
  const uint16_t lo = f2bf(d2);
  res = d2 - bf2f(lo);
  return lo;
}
// the row bound from the fp32 sum of squared residuals (lo16_elem) and the fp64 norm of x (1 after normalising)
__device__ __forceinline__ float lo16_bound(double ss_res) {
  return f32_round_up(sqrt(ss_res) * (1.0 + 1e-4) + 5.9605e-8 * (1.0 + 1e-6) + 1e-12);
}
// fp16 of a normalised element through fp32 (v_cvt_f32_f64 then v_cvt_f16_f32).  The fp32 value is made opaque
// so the compiler keeps the two hardware conversions: it otherwise folds them into ONE fp64 -> fp16 conversion,
// which gfx950 has no instruction for and which it expands into ~25 integer / compare instructions per element
// (the bound is computed from the value stored either way)
__device__ __forceinline__ _Float16 f16_via_f32(double xh, float& xf) {
  xf = (float)xh;
  asm volatile("" : "+v"(xf));
  return (_Float16)xf;
}

__device__ __forceinline__ void pack_elem(double xh, bool want_f16, uint16_t& h, uint16_t& l, uint16_t& f,
                                          PackAcc& acc) {
  float xf;
  const _Float16 hf16 = f16_via_f32(xh, xf);
  if (want_f16) {
    const double r3 = xh - (double)hf16;
    acc.e3 = fma(r3, r3, acc.e3);
    f = __builtin_bit_cast(uint16_t, hf16);
  }
  h = f2bf(xf);
  const float hf = bf2f(h);
  l = f2bf(xf - hf);
  const double r1 = xh - (double)hf;
  const double r2 = r1 - (double)bf2f(l);
  acc.e1 = fma(r1, r1, acc.e1);
  acc.e2 = fma(r2, r2, acc.e2);
}

typedef unsigned short cmve_u16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t cmve_u32x2 __attribute__((ext_vector_type(2)));

// zero planes of a padding row (d_pad % 64 == 0)
__device__ __forceinline__ void pack_pad_row(uint16_t* hrow, uint16_t* lrow, uint16_t* frow, int64_t d_pad,
                                             int lane) {
  const cmve_u16x4 z = {0, 0, 0, 0};
  for (int64_t k = (int64_t)lane * 4; k < d_pad; k += 256) {
    gst((cmve_u16x4*)(hrow + k), z);
    if (lrow) gst((cmve_u16x4*)(lrow + k), z);
    if (frow) gst((cmve_u16x4*)(frow + k), z);
  }
}

// pack one row x * inv into the planes (lrow / frow nullable); b1/b2/b3 = rigorous residual bounds of
// hi, hi+lo and f16 (wave-uniform)
template <typename T>
__device__ __forceinline__ void pack_row_planes(const T* __restrict__ x, int64_t d, int64_t d_pad, bool vec,
                                                double inv, uint16_t* hrow, uint16_t* lrow, uint16_t* frow,
                                                int lane, float& b1, float& b2, float& b3) {
  const bool want_f16 = frow != nullptr;
  PackAcc acc;
  bool done = false;
  if (vec) {  // rows_vec4: 16-B loads, four elements per lane step, 8-B plane stores
    for (int64_t k = (int64_t)lane * 4; k < d_pad; k += 256) {
      cmve_u16x4 hv = {0, 0, 0, 0}, lv = {0, 0, 0, 0}, fv = {0, 0, 0, 0};
      if (k < d) {  // d % 4 == 0: all four valid
        double e[4];
        load4d(x + k, e);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          uint16_t h, l, f = 0;
          pack_elem(e[c] * inv, want_f16, h, l, f, acc);
          hv[c] = h;
          lv[c] = l;
          fv[c] = f;
        }
      }
      *(cmve_u16x4*)(hrow + k) = hv;
      if (lrow) *(cmve_u16x4*)(lrow + k) = lv;
      if (frow) *(cmve_u16x4*)(frow + k) = fv;
    }
    done = true;
  }
  if (!done)
    for (int64_t k = lane; k < d_pad; k += WAVE) {
      uint16_t h = 0, l = 0, f = 0;
      if (k < d) pack_elem((double)x[k] * inv, want_f16, h, l, f, acc);
      hrow[k] = h;
      if (lrow) lrow[k] = l;
      if (frow) frow[k] = f;
    }
  const double e1 = wave_sum(acc.e1), e2 = wave_sum(acc.e2), e3 = wave_sum(acc.e3);
  // sqrt rounding + the fp64 error of x*inv itself (~1e-16 per element) -> small slack
  b1 = f32_round_up(sqrt(e1) * (1.0 + 1e-9) + 1e-12);
  b2 = f32_round_up(sqrt(e2) * (1.0 + 1e-9) + 1e-12);
  b3 = f32_round_up(sqrt(e3) * (1.0 + 1e-9) + 1e-12);
}

// 1-based GT rank from a better-than-GT count (LINAS-engine/util/metrics.py:137-147): sgt NaN (empty
// GT list) -> n_m + 1 (metrics.py:140); sgt +inf (every GT scores NaN) -> n_m (np.argsort puts NaN
// after every finite score; numpy's order among several NaN is implementation-defined: the GT is
// taken as the last); else count + 1
__device__ __forceinline__ int64_t gt_rank_of(int32_t cnt, double sgt, int64_t n_m) {
  return (sgt != sgt) ? n_m + 1 : (sgt == (double)INFINITY ? n_m : (int64_t)cnt + 1);
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
constexpr int EVAL_EMAX_SHARDS = 64;  // K14: err_max shards per side and plane (eval.hip, sim.hip)

// canonical exact score: cos64(x, y) = dot64(raw_x, raw_y) * (inv_x * inv_y), symmetric in (x, y), so
// the GT-score, fix-up and top-k re-score kernels score a pair bit-identically
template <typename TA, typename TB, bool LIGHT = false>
__device__ __forceinline__ double wave_cos64(const TA* xa, const TB* xb, double inva, double invb, int64_t d,
                                             int lane) {
  return wave_dot64<TA, TB, LIGHT>(xa, xb, d, lane) * (inva * invb);
}

// ---- K14 level-2 re-score: one pair's score from the fp16 + bf16 residual planes (lo16_elem, cmve_internal.h) ----
// lane L holds elements [16L, 16L + 16) of each 1024-element chunk: two 16-B fp16 loads and two 16-B bf16 loads
// per row and chunk.  x2 = h + lo is formed in fp64 (exact unless lo lies 2^-42 below h: then within 2^-53 |x2|),
// the products and sums in fp64, so the sum's error is a few ulps of 1:
//   |s2 - cos64| <= el_q + (1 + el_q) el_g + 2e-12
// (the 2e-12 covers the fp64 sums here and in cos64, as score_error_bound's 1e-12 does for the MFMA bound)
typedef uint32_t cmve_u32x4 __attribute__((ext_vector_type(4)));
struct L16Frag {
  cmve_u32x4 h0, h1, l0, l1;
};
__device__ __forceinline__ void l16_load(const uint16_t* __restrict__ hrow, const uint16_t* __restrict__ lrow,
                                         int64_t k, L16Frag& f) {
  f.h0 = gld((const cmve_u32x4*)(hrow + k));
  f.h1 = gld((const cmve_u32x4*)(hrow + k + 8));
  f.l0 = gld((const cmve_u32x4*)(lrow + k));
  f.l1 = gld((const cmve_u32x4*)(lrow + k + 8));
}
__device__ __forceinline__ double l16_x(uint32_t hw, uint32_t lw, int half) {
  const uint16_t h = (uint16_t)(hw >> (16 * half));
  const uint32_t l = half ? (lw & 0xffff0000u) : (lw << 16);
  return (double)(float)__builtin_bit_cast(_Float16, h) + (double)__uint_as_float(l);
}
__device__ __forceinline__ double l16_partial(const L16Frag& a, const L16Frag& b, double acc) {
  const uint32_t ah[8] = {a.h0.x, a.h0.y, a.h0.z, a.h0.w, a.h1.x, a.h1.y, a.h1.z, a.h1.w};
  const uint32_t al[8] = {a.l0.x, a.l0.y, a.l0.z, a.l0.w, a.l1.x, a.l1.y, a.l1.z, a.l1.w};
  const uint32_t bh[8] = {b.h0.x, b.h0.y, b.h0.z, b.h0.w, b.h1.x, b.h1.y, b.h1.z, b.h1.w};
  const uint32_t bl[8] = {b.l0.x, b.l0.y, b.l0.z, b.l0.w, b.l1.x, b.l1.y, b.l1.z, b.l1.w};
#pragma unroll
  for (int e = 0; e < 16; ++e)
    acc = fma(l16_x(ah[e >> 1], al[e >> 1], e & 1), l16_x(bh[e >> 1], bl[e >> 1], e & 1), acc);
  return acc;
}
// XCD-ordered re-score of the bucketed undecided pairs: XCD x (blockIdx & 7) owns buckets
// x, x+8, ...; its waves stride through those buckets' pairs in order, so at any time an XCD works
// on one or two buckets and their raw gallery rows (1 MiB each) stay in its L2.
// PREFETCH: load the pair's GT scores before its dot product (latency-bound small evaluations; in the
// bandwidth-bound bench-size fix-up that was 3% slower)
// flat: one group over all buckets and every wave of the grid (small evaluations: a 1k-row gallery has
// 4 buckets, which the XCD grouping would leave to 4 of the 8 XCDs); the caller keeps nb <= 4096
// the exclusive prefix of the bucket sizes a fix-up walks (wave 0 of the block): buckets xcd, xcd + G, ..., nk
// of them, each clamped to cap_b; pre[nk] = the total (lane-chunked sums + a wave scan)
__device__ __forceinline__ void fixup_prefix(const uint64_t* __restrict__ cand, int64_t nb, int64_t cap_b, int xcd,
                                             int G, int64_t nk, int lane, int64_t* pre) {
  const int64_t per = (nk + 63) / 64;
  const int64_t k0 = lane * per, k1 = min(nk, k0 + per);
  if (per <= 4) {  // (<= 256 buckets: one round of loads held in registers)
    int64_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (k0 + j < k1) ? min((int64_t)gld(cand + xcd + G * (k0 + j)), cap_b) : 0;
    const int64_t sum = (v[0] + v[1]) + (v[2] + v[3]);
    int64_t incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    int64_t run = incl - sum;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (k0 + j < k1) {
        pre[k0 + j] = run;
        run += v[j];
      }
    if (lane == 63) pre[nk] = incl;
  } else {
    int64_t sum = 0;
    for (int64_t k = k0; k < k1; ++k) sum += min((int64_t)gld(cand + xcd + G * k), cap_b);
    int64_t incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    int64_t run = incl - sum;
    for (int64_t k = k0; k < k1; ++k) {
      pre[k] = run;
      run += min((int64_t)gld(cand + xcd + G * k), cap_b);
    }
    if (lane == 63) pre[nk] = incl;
  }
}

// DYN_PRE: the bucket prefix in dynamic LDS sized by the launch ((buckets per group + 1) * 8 bytes) instead of the
// 32 KiB static array, which capped the fix-up at 5 blocks per CU whatever its registers allowed
template <typename TQ, typename TG, bool PREFETCH = false, bool DYN_PRE = false, bool LIGHT = false>
__device__ __forceinline__ void fixup_walk(const TQ* __restrict__ qraw, int64_t ldq,
                                                    const double* __restrict__ qinv, const TG* __restrict__ graw,
                                                    int64_t ldg, const double* __restrict__ ginv, int64_t d,
                                                    const double* __restrict__ row_sgt,
                                                    const double* __restrict__ col_sgt, int* __restrict__ row_cnt,
                                                    int* __restrict__ col_cnt, const uint64_t* __restrict__ cand,
                                                    int64_t nb, int64_t cap_b, bool flat = false) {
  int64_t* pre;
  if constexpr (DYN_PRE) {
    extern __shared__ int64_t fix_dyn_pre[];
    pre = fix_dyn_pre;
  } else {
    __shared__ int64_t fix_pre[FIXUP_MAX_BUCKETS_PER_XCD + 1];
    pre = fix_pre;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int G = flat ? 1 : 8;  // bucket groups (XCDs)
  const int xcd = flat ? 0 : (blockIdx.x & 7);
  const int64_t nk = xcd < nb ? (nb - xcd + G - 1) / G : 0;
  if (wave == 0) fixup_prefix(cand, nb, cap_b, xcd, G, nk, lane, pre);
  __syncthreads();
  const int64_t total = pre[nk];
  const int nw = (int)(blockDim.x >> 6);  // waves per block
  const int64_t stride = (int64_t)(gridDim.x / G) * nw;
  int64_t k = 0;
  auto entry = [&](int64_t cc) -> uint64_t {  // pair cc's entry (cc increases call by call); 0 past the end
    if (cc >= total) return 0ull;
    if (pre[k + 1] <= cc) {  // the bucket holding pair cc: binary search of the prefix (the flat walk of
      int64_t lo = k + 1, hi = nk - 1;  // a 256-bucket evaluation would scan up to 256 LDS words)
      while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= cc) lo = mid;
        else hi = mid - 1;
      }
      k = lo;
    }
    return gld(cand + nb + (xcd + G * k) * cap_b + (cc - pre[k]));
  };
  // the next pair's entry is loaded one pair ahead: in flight with this pair's row loads (as a dependent load
  // at the top of each pair it added a round trip to every pair)
  const int64_t c0 = (int64_t)(blockIdx.x / G) * nw + wave;
  uint64_t u_next = entry(c0);
  for (int64_t c = c0; c < total;) {
    const uint64_t u = u_next;
    c += stride;
    u_next = entry(c);
    const int64_t i = (int64_t)(u & 0x7fffffffull);
    const int64_t j = (int64_t)((u >> 31) & 0x7fffffffull);
    uint32_t flags = (uint32_t)(u >> 62);
    if (!flags) continue;  // (a null entry)
    double rs = 0.0, cs = 0.0;
    if (PREFETCH) {
      rs = ((flags & 1u) && row_sgt) ? gld(row_sgt + i) : 0.0;
      cs = ((flags & 2u) && col_sgt) ? gld(col_sgt + j) : 0.0;
    }
    const double s = wave_cos64<TQ, TG, LIGHT>(qraw + i * ldq, graw + j * ldg, gld(qinv + i), gld(ginv + j), d, lane);
    if (lane == 0) {
      if ((flags & 1u) && row_sgt && s > (PREFETCH ? rs : gld(row_sgt + i))) gadd(row_cnt + i, 1);
      if ((flags & 2u) && col_sgt && s > (PREFETCH ? cs : gld(col_sgt + j))) gadd(col_cnt + j, 1);
    }
  }
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
