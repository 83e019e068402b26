// K14: one exact two-direction GT-rank evaluation of a resident problem in three launches
// (cmve_eval_ranks, host side in sim.hip):
//   1. eval_prep_kernel  K1 pack of BOTH sets, the exact fp64 GT score of every row of both
//                        directions (K5a) and zeroed counters; the LAST block to finish derives the
//                        sets' err_max and every rank threshold (agent-scope release / acquire
//                        hand-off, cdna_hip_programming.md Guideline 16)
//   2. sim_kernel<RANK>  K4 rank GEMM (certain counts + undecided pairs), unchanged
//   3. eval_fix_kernel   K5b fp64 re-score of the undecided pairs; the LAST block turns the counts into
//                        1-based ranks, R@1/5/10 + rank sums per direction, the pair total and the
//                        overflow size
// It replaces the per-evaluation chain of the reference's validation / test loop
// (LINAS-engine/validate.py:61-74, tester.py:133-139): evaluation.cal_error (evaluation.py:17-21,
// both sets re-normalised, the full matrix in fp64) -> util/metrics.eval_q2m in both directions
// (metrics.py:124-157, an argsort per row).  The separate-launch path (cmve_pack_rows x2,
// cmve_gt_thresholds x2, cmve_rank_count, cmve_gt_ranks x2) computes the identical numbers: the
// pack, GT-score and fix-up arithmetic are the same device functions (cmve_internal.h).
#include "eval_abi.h"

namespace cmve {

__device__ __forceinline__ const float* side_err(const EvalSide& s, int mode) {
  return mode == CMVE_SIM_BF16 ? s.err_hi : (mode == CMVE_SIM_BF16X3 ? s.err_hilo : s.err_h16);
}

// ---- in-launch hand-off to the last block (MI355X_MICROARCH.md "inter-workgroup visibility", valid form
// "ONE lane of each storing workgroup ... agent-scope atomic add ... the workgroup whose add came last"):
// the handed-off words are stored write-through (sc1: agent-scope relaxed atomic stores) or are agent
// atomics, every wave waits for them (vmcnt(0)) before the block's barrier, one lane adds to the
// arrival counter, and the last block reads them with sc1 loads behind one acquire.  No per-block L2
// write-back (an agent release per block cost ~40 us over 512 blocks that had just dirtied the planes).
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) int gi32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
// (integer atomics: ROCm 7.2 lowered a relaxed agent-scope atomic store of a float / double to a
// plain global_store, without sc1)
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((gu64*)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store((gu32*)p, __builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __builtin_bit_cast(float, __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ int ld_sc1(const int* p) {
  return __hip_atomic_load((gi32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_sc1(const unsigned long long* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Arrival counting in two levels: block b adds to shard counter 1 + b % ARR_SHARDS (each on a line of
// its own); the block completing a shard adds to the top counter 0, and the block completing the top
// counter is the last.  One same-address atomic per block serialises at one L2 channel (~30 ns each:
// 512 arrivals cost ~15 us), the shards take them in parallel.  Each block's handed-off words are
// sc1 stores or agent atomics that completed (vmcnt(0)) before its add; the adds chain causally to
// the last block, which reads them with sc1 loads behind one acquire.  The completing blocks reset the
// counters they completed, so the words are zero again for the next launch (zeroed at allocation).
constexpr int ARR_SHARDS = 8, ARR_STRIDE = 64;  // counters 256 B apart
__device__ __forceinline__ bool last_block_arrival(unsigned* ctr_flat) {
  __shared__ int s_last;
  gu32* ctr = (gu32*)ctr_flat;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its sc1 stores / atomics have completed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned b = blockIdx.x, G = gridDim.x, sh = b % ARR_SHARDS;
    const unsigned shard_size = (G - sh + ARR_SHARDS - 1) / ARR_SHARDS;
    const unsigned shards = G < (unsigned)ARR_SHARDS ? G : (unsigned)ARR_SHARDS;
    gu32* sc = ctr + ARR_STRIDE * (1 + sh);
    int last = 0;
    if (__hip_atomic_fetch_add(sc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == shard_size - 1) {
      __hip_atomic_store(sc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == shards - 1) {
        __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = 1;
      }
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return false;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return true;
}

// prep_row for rows of <= 1024 elements that both sides read in 16-B pieces (rows_vec4): the row is
// loaded ONCE into registers (16 doubles per lane, elements 4L + 256m + c) and packed from there, and
// each GT partner is read once for both its sum of squares and the dot product.  Every per-lane
// accumulation runs in the (m, c) order of row_sumsq / pack_row_planes / wave_dot64, so the planes,
// bounds, norms and GT scores are bit-identical to the streaming path (and to cmve_pack_rows /
// cmve_gt_thresholds).
template <typename TA, typename TB>
__device__ __forceinline__ void prep_row_regs(const EvalSide& A, const EvalSide& B, const EvalCommon& c, int64_t row,
                                              const TA* __restrict__ x, uint16_t* hrow, uint16_t* lrow,
                                              uint16_t* frow, int lane) {
  double v[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int64_t k = (int64_t)lane * 4 + 256 * m;
    if (k < c.d) load4d(x + k, v[m]);
    else v[m][0] = v[m][1] = v[m][2] = v[m][3] = 0.0;
  }
  double ss = 0.0;
#pragma unroll
  for (int m = 0; m < 4; ++m)
    if ((int64_t)lane * 4 + 256 * m < c.d)
#pragma unroll
      for (int q = 0; q < 4; ++q) ss = fma(v[m][q], v[m][q], ss);
  const double inv = row_inv_norm(wave_sum(ss), A.eps, A.flags);
  const bool want_f16 = frow != nullptr;
  PackAcc acc;
  if (c.mode == CMVE_SIM_F16 && want_f16) {
    // the F16 rank GEMM reads only the fp16 plane: the bf16 planes are not written and their bounds
    // are +inf (a stale plane can never pass for a bounded one)
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int64_t k = (int64_t)lane * 4 + 256 * m;
      if (k >= c.d_pad) break;
      cmve_u16x4 fv = {0, 0, 0, 0};
      if (k < c.d) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const double xh = v[m][q] * inv;
          const _Float16 hf16 = (_Float16)(float)xh;  // pack_elem's f16 arithmetic
          const double r3 = xh - (double)hf16;
          acc.e3 = fma(r3, r3, acc.e3);
          fv[q] = __builtin_bit_cast(uint16_t, hf16);
        }
      }
      *(cmve_u16x4*)(frow + k) = fv;
    }
  } else {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int64_t k = (int64_t)lane * 4 + 256 * m;
      if (k >= c.d_pad) break;
      cmve_u16x4 hv = {0, 0, 0, 0}, lv = {0, 0, 0, 0}, fv = {0, 0, 0, 0};
      if (k < c.d) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint16_t h, l, f = 0;
          pack_elem(v[m][q] * inv, want_f16, h, l, f, acc);
          hv[q] = h;
          lv[q] = l;
          fv[q] = f;
        }
      }
      *(cmve_u16x4*)(hrow + k) = hv;
      if (lrow) *(cmve_u16x4*)(lrow + k) = lv;
      if (frow) *(cmve_u16x4*)(frow + k) = fv;
    }
  }
  const bool bf = !(c.mode == CMVE_SIM_F16 && want_f16);
  const double e1 = bf ? wave_sum(acc.e1) : 0.0, e2 = bf ? wave_sum(acc.e2) : 0.0, e3 = wave_sum(acc.e3);
  if (lane == 0) {
    A.inv[row] = inv;
    // pack_row_planes' bounds
    st_sc1(&A.err_hi[row], bf ? f32_round_up(sqrt(e1) * (1.0 + 1e-9) + 1e-12) : INFINITY);
    st_sc1(&A.err_hilo[row], bf ? f32_round_up(sqrt(e2) * (1.0 + 1e-9) + 1e-12) : INFINITY);
    if (A.err_h16) st_sc1(&A.err_h16[row], f32_round_up(sqrt(e3) * (1.0 + 1e-9) + 1e-12));
  }
  if (!A.off) return;
  double best = -INFINITY;
  bool any = false;
  for (int64_t g = A.off[row]; g < A.off[row + 1]; ++g) {
    const TB* y = (const TB*)B.raw + (int64_t)A.idx[g] * B.ld;
    double w[4][4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int64_t k = (int64_t)lane * 4 + 256 * m;
      if (k < c.d) load4d(y + k, w[m]);
    }
    double dot = 0.0, yy = 0.0;
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if ((int64_t)lane * 4 + 256 * m < c.d)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          dot = fma(v[m][q], w[m][q], dot);
          yy = fma(w[m][q], w[m][q], yy);
        }
    const double invb = row_inv_norm(wave_sum(yy), B.eps, B.flags);
    const double s = wave_sum(dot) * (inv * invb);  // wave_cos64(x, y, inv, invb)
    if (s == s) {
      any = true;
      if (s > best) best = s;
    }
  }
  if (lane == 0) {
    st_sc1(&A.sgt[row], any ? best : (A.off[row + 1] > A.off[row] ? (double)INFINITY : (double)NAN));
    A.cnt[row] = 0;
  }
}

// pack row `row` of side A and score its GT list against side B (one wave)
template <typename TA, typename TB>
__device__ __forceinline__ void prep_row(const EvalSide& A, const EvalSide& B, const EvalCommon& c, int64_t row,
                                         int lane) {
  uint16_t* hrow = A.hi + row * c.d_pad;
  uint16_t* lrow = A.lo ? A.lo + row * c.d_pad : nullptr;
  uint16_t* frow = A.h16 ? A.h16 + row * c.d_pad : nullptr;
  if (row >= A.n) {  // padding rows: zero vectors, zero bounds, never counted
    pack_pad_row(hrow, lrow, frow, c.d_pad, lane);
    if (lane == 0) {
      A.inv[row] = 0.0;
      st_sc1(&A.err_hi[row], 0.f);
      st_sc1(&A.err_hilo[row], 0.f);
      if (A.err_h16) st_sc1(&A.err_h16[row], 0.f);
      if (A.off) {
        st_sc1(&A.sgt[row], (double)NAN);
        A.cnt[row] = 0;
      }
    }
    return;
  }
  const TA* x = (const TA*)A.raw + row * A.ld;
  if (A.vec && B.vec && c.d_pad <= 1024) {
    prep_row_regs<TA, TB>(A, B, c, row, x, hrow, lrow, frow, lane);
    return;
  }
  const double inv = row_inv_norm(row_sumsq<TA>(x, c.d, A.vec != 0, lane), A.eps, A.flags);
  float b1, b2, b3;
  pack_row_planes<TA>(x, c.d, c.d_pad, A.vec != 0, inv, hrow, lrow, frow, lane, b1, b2, b3);
  if (lane == 0) {
    A.inv[row] = inv;
    st_sc1(&A.err_hi[row], b1);  // handed to the last block (sc1): the rest only to later launches
    st_sc1(&A.err_hilo[row], b2);
    if (A.err_h16) st_sc1(&A.err_h16[row], b3);
  }
  if (!A.off) return;
  // exact GT score (gt_thr_kernel's arithmetic): the partner's 1/||y|| is recomputed by the routine
  // that packs it, so it equals the partner's stored inv_norm bit for bit
  double best = -INFINITY;
  bool any = false;
  for (int64_t k = A.off[row]; k < A.off[row + 1]; ++k) {
    const int64_t b = A.idx[k];
    const TB* y = (const TB*)B.raw + b * B.ld;
    const double invb = row_inv_norm(row_sumsq<TB>(y, c.d, B.vec != 0, lane), B.eps, B.flags);
    const double s = wave_cos64(x, y, inv, invb, c.d, lane);
    if (s == s) {
      any = true;
      if (s > best) best = s;
    }
  }
  if (lane == 0) {
    // empty list: NaN (rank n_m + 1); every GT NaN: +inf (rank n_m) -- gt_thr_kernel's encoding
    st_sc1(&A.sgt[row], any ? best : (A.off[row + 1] > A.off[row] ? (double)INFINITY : (double)NAN));
    A.cnt[row] = 0;
  }
}

constexpr int EVAL_NT = 1024;  // threads per block of both kernels: the last block's tail covers a
                               // 1k-row side in one pass
constexpr int EVAL_NW = EVAL_NT / 64;

// reduce K values per thread over the block in ONE LDS round (max or sum); every thread gets the K
// results in v (a reduction per value cost two barriers each: ~0.5 us per value in the tail)
template <bool MAX, typename T, int K>
__device__ __forceinline__ void block_reduce_k(T (&v)[K], T* red /* LDS [K + 1][EVAL_NW] */) {
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const T u = __shfl_xor(v[k], o, 64);
      v[k] = MAX ? (u > v[k] ? u : v[k]) : v[k] + u;
    }
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) red[k * EVAL_NW + (threadIdx.x >> 6)] = v[k];
  __syncthreads();
  T* out = red + K * EVAL_NW;  // thread k < K folds row k (wave order: deterministic)
  if (threadIdx.x < K) {
    const T* r = red + threadIdx.x * EVAL_NW;
    T a = r[0];
#pragma unroll
    for (int w = 1; w < EVAL_NW; ++w) a = MAX ? (r[w] > a ? r[w] : a) : a + r[w];
    out[threadIdx.x] = a;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = out[k];
}

// The last block of the prep launch: err_max of both sides (all three planes, real rows, NaN skipped:
// err_max_kernel's result) and every rank threshold (gt_thr_kernel's).  Each pass issues all of a
// thread's loads before using them (the tail runs on one CU: its latency is the launch's).
__device__ __forceinline__ void prep_tail(const EvalSide& q, const EvalSide& g, const EvalCommon& c) {
  __shared__ float red[7 * EVAL_NW];
  float m[2][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
  const int64_t nmax = q.n > g.n ? q.n : g.n;
  for (int64_t i = threadIdx.x; i < nmax; i += EVAL_NT) {
    float e[2][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    if (i < q.n) {
      e[0][0] = ld_sc1(&q.err_hi[i]);
      e[0][1] = ld_sc1(&q.err_hilo[i]);
      if (q.err_h16) e[0][2] = ld_sc1(&q.err_h16[i]);
    }
    if (i < g.n) {
      e[1][0] = ld_sc1(&g.err_hi[i]);
      e[1][1] = ld_sc1(&g.err_hilo[i]);
      if (g.err_h16) e[1][2] = ld_sc1(&g.err_h16[i]);
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int k = 0; k < 3; ++k) m[s2][k] = fmaxf(m[s2][k], e[s2][k]);  // fmaxf drops a NaN operand
  }
  float mm[6] = {m[0][0], m[0][1], m[0][2], m[1][0], m[1][1], m[1][2]};
  block_reduce_k<true>(mm, red);
  if (threadIdx.x < 3) {
    q.err_max[threadIdx.x] = mm[threadIdx.x];
    g.err_max[threadIdx.x] = mm[3 + threadIdx.x];
  }
  const int slot = mode_slot(c.mode);
  const float qmax = mm[slot], gmax = mm[3 + slot];
  const float* qerr = side_err(q, c.mode);
  const float* gerr = side_err(g, c.mode);
  const int64_t pmax = q.n_pad > g.n_pad ? q.n_pad : g.n_pad;
  for (int64_t r = threadIdx.x; r < pmax; r += EVAL_NT) {
    const bool dq = q.off && r < q.n_pad, dg = g.off && r < g.n_pad;
    double sq = 0.0, sg = 0.0;
    float eq = 0.f, eg = 0.f;
    if (dq) {
      sq = ld_sc1(&q.sgt[r]);
      eq = ld_sc1(&qerr[r]);
    }
    if (dg) {
      sg = ld_sc1(&g.sgt[r]);
      eg = ld_sc1(&gerr[r]);
    }
    // NaN (no GT, padding) or +inf (every GT NaN): never counted
    if (dq) {
      const double E = score_error_bound((double)eq, (double)gmax, c.d_pad, c.mode);
      q.thr_hi[r] = sq < INFINITY ? f32_round_up(sq + E) : INFINITY;
      q.thr_lo[r] = sq < INFINITY ? f32_round_down(sq - E) : INFINITY;
    }
    if (dg) {
      const double E = score_error_bound((double)eg, (double)qmax, c.d_pad, c.mode);
      g.thr_hi[r] = sg < INFINITY ? f32_round_up(sg + E) : INFINITY;
      g.thr_lo[r] = sg < INFINITY ? f32_round_down(sg - E) : INFINITY;
    }
  }
}

template <typename TQ, typename TG>
__global__ __launch_bounds__(EVAL_NT) void eval_prep_kernel(EvalSide q, EvalSide g, EvalCommon c) {
  EVAL_STAMP(c, 0, 0);
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * EVAL_NW + (threadIdx.x >> 6);
  for (int64_t t = (int64_t)blockIdx.x * EVAL_NT + threadIdx.x; t < c.nb; t += (int64_t)gridDim.x * EVAL_NT)
    c.bucket[t] = 0;
  if (!(c.dbg & 1)) {
    if (row < q.n_pad)
      prep_row<TQ, TG>(q, g, c, row, lane);
    else if (row < q.n_pad + g.n_pad)
      prep_row<TG, TQ>(g, q, c, row - q.n_pad, lane);
  }
  EVAL_STAMP(c, 0, 1);
  if (c.dbg & 2) return;
  if (!last_block_arrival(c.done)) return;
  EVAL_STAMP(c, 0, 2);
  if (c.dbg & 4) return;
  prep_tail(q, g, c);
  EVAL_STAMP(c, 0, 3);
}

// The last block of the fix-up launch: pair total / overflow size (cand_finalize_kernel's), the ranks
// of both directions (cmve_gt_ranks' rules) and per direction #rank<=1, <=5, <=10 and the rank sum.
__device__ __forceinline__ void fix_tail(const EvalSide& q, const EvalSide& g, const EvalCommon& c) {
  __shared__ unsigned long long red[10 * EVAL_NW];
  __shared__ unsigned long long redm[2 * EVAL_NW];
  unsigned long long tot = 0, mx = 0;
  for (int64_t b = threadIdx.x; b < c.nb; b += EVAL_NT) {
    const unsigned long long v = ld_sc1(&c.bucket[b]);
    tot += v;
    mx = v > mx ? v : mx;
  }
  unsigned long long acc[2][4] = {};
  const int64_t nmax = q.n > g.n ? q.n : g.n;
  for (int64_t i = threadIdx.x; i < nmax; i += EVAL_NT) {
    const bool dq = q.off && i < q.n, dg = g.off && i < g.n;
    int32_t cq = 0, cg = 0;
    double sq = 0.0, sg = 0.0;
    if (dq) {
      cq = ld_sc1(&q.cnt[i]);  // agent atomics of this launch and the GEMM's
      sq = q.sgt[i];           // written by an earlier launch
    }
    if (dg) {
      cg = ld_sc1(&g.cnt[i]);
      sg = g.sgt[i];
    }
    if (dq) {
      const int64_t r = gt_rank_of(cq, sq, g.n);
      q.ranks[i] = r;
      acc[0][0] += (r <= 1);
      acc[0][1] += (r <= 5);
      acc[0][2] += (r <= 10);
      acc[0][3] += (unsigned long long)r;
    }
    if (dg) {
      const int64_t r = gt_rank_of(cg, sg, q.n);
      g.ranks[i] = r;
      acc[1][0] += (r <= 1);
      acc[1][1] += (r <= 5);
      acc[1][2] += (r <= 10);
      acc[1][3] += (unsigned long long)r;
    }
  }
  unsigned long long sums[9] = {acc[0][0], acc[0][1], acc[0][2], acc[0][3], acc[1][0], acc[1][1], acc[1][2],
                                acc[1][3], tot};
  unsigned long long mxs[1] = {mx};
  block_reduce_k<false>(sums, red);
  block_reduce_k<true>(mxs, redm);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < 4 ? q.off : g.off) c.stats[k] = (int64_t)sums[k];
    c.stats[8] = (int64_t)sums[8];
    c.stats[9] = (int64_t)mxs[0] > c.cap_b ? ((int64_t)mxs[0] + 1) * c.nb + c.nb + 1 : 0;
  }
}

template <typename TQ, typename TG>
__global__ __launch_bounds__(EVAL_NT) void eval_fix_kernel(EvalSide q, EvalSide g, EvalCommon c) {
  EVAL_STAMP(c, 2, 0);
  if (!(c.dbg & 8))
    fixup_walk<TQ, TG, true>((const TQ*)q.raw, q.ld, q.inv, (const TG*)g.raw, g.ld, g.inv, c.d, q.off ? q.sgt : nullptr,
                       g.off ? g.sgt : nullptr, q.cnt, g.cnt, c.cand, c.nb, c.cap_b);
  EVAL_STAMP(c, 2, 1);
  if (c.dbg & 16) return;
  if (!last_block_arrival(c.done + EVAL_ARRIVAL_WORDS)) return;
  EVAL_STAMP(c, 2, 2);
  if (c.dbg & 32) return;
  fix_tail(q, g, c);
  EVAL_STAMP(c, 2, 3);
}

template <typename TQ, typename TG>
static int launch_eval_typed(const EvalSide& q, const EvalSide& g, const EvalCommon& c, int phase, hipStream_t s) {
  if (phase == 0) {
    const unsigned blocks = (unsigned)((q.n_pad + g.n_pad + EVAL_NW - 1) / EVAL_NW);
    hipLaunchKernelGGL((eval_prep_kernel<TQ, TG>), dim3(blocks), dim3(EVAL_NT), 0, s, q, g, c);
    return check_launch("eval_prep_kernel");
  }
  // 16 blocks of 16 waves per XCD: 2,048 waves for the few thousand undecided pairs of an evaluation
  // of this size (the rank fix-up's grid is sized for millions of pairs)
  hipLaunchKernelGGL((eval_fix_kernel<TQ, TG>), dim3(8u * 16u), dim3(EVAL_NT), 0, s, q, g, c);
  return check_launch("eval_fix_kernel");
}

// phase 0: prep, phase 1: fix-up + ranks
int launch_eval(const EvalSide& q, const EvalSide& g, const EvalCommon& c, int q_f64, int g_f64, int phase,
                hipStream_t s) {
  if (!q_f64 && !g_f64) return launch_eval_typed<float, float>(q, g, c, phase, s);
  if (!q_f64 && g_f64) return launch_eval_typed<float, double>(q, g, c, phase, s);
  if (q_f64 && !g_f64) return launch_eval_typed<double, float>(q, g, c, phase, s);
  return launch_eval_typed<double, double>(q, g, c, phase, s);
}

}  // namespace cmve
