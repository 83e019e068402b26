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
      A.err_hi[row] = 0.f;
      A.err_hilo[row] = 0.f;
      if (A.err_h16) A.err_h16[row] = 0.f;
      if (A.off) {
        A.sgt[row] = NAN;
        A.cnt[row] = 0;
      }
    }
    return;
  }
  const TA* x = (const TA*)A.raw + row * A.ld;
  const double inv = row_inv_norm(row_sumsq<TA>(x, c.d, A.vec != 0, lane), A.eps, A.flags);
  float b1, b2, b3;
  pack_row_planes<TA>(x, c.d, c.d_pad, A.vec != 0, inv, hrow, lrow, frow, lane, b1, b2, b3);
  if (lane == 0) {
    A.inv[row] = inv;
    A.err_hi[row] = b1;
    A.err_hilo[row] = b2;
    if (A.err_h16) A.err_h16[row] = b3;
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
    A.sgt[row] = any ? best : (A.off[row + 1] > A.off[row] ? (double)INFINITY : (double)NAN);
    A.cnt[row] = 0;
  }
}

// max of the per-row bounds of a side's three planes over its real rows (err_max_kernel: NaN skipped),
// stored to s.err_max and returned in out[0..3) (LDS: the stored words are not re-read through the
// scalar cache, which vector stores do not update)
__device__ __forceinline__ void block_err_max(const EvalSide& s, float* red /* LDS [3][4] */, float* out) {
  float m0 = 0.f, m1 = 0.f, m2 = 0.f;
  for (int64_t i = threadIdx.x; i < s.n; i += 256) {
    m0 = fmaxf(m0, s.err_hi[i]);
    m1 = fmaxf(m1, s.err_hilo[i]);
    if (s.err_h16) m2 = fmaxf(m2, s.err_h16[i]);
  }
  m0 = wave_max(m0);
  m1 = wave_max(m1);
  m2 = wave_max(m2);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w] = m0;
    red[4 + w] = m1;
    red[8 + w] = m2;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const float* r = red + 4 * threadIdx.x;
    const float m = fmaxf(fmaxf(r[0], r[1]), fmaxf(r[2], r[3]));
    s.err_max[threadIdx.x] = m;
    out[threadIdx.x] = m;
  }
  __syncthreads();
}

// thresholds of side A's rows against side B's error bound (gt_thr_kernel / thr_from_sgt_kernel)
__device__ __forceinline__ void side_thresholds(const EvalSide& A, float bmax, const EvalCommon& c) {
  const float* aerr = side_err(A, c.mode);
  for (int64_t r = threadIdx.x; r < A.n_pad; r += 256) {
    const double s = A.sgt[r];
    if (!(s < INFINITY)) {  // NaN (no GT, padding) or +inf (every GT NaN): never counted
      A.thr_hi[r] = INFINITY;
      A.thr_lo[r] = INFINITY;
    } else {
      const double E = score_error_bound((double)aerr[r], (double)bmax, c.d_pad, c.mode);
      A.thr_hi[r] = f32_round_up(s + E);
      A.thr_lo[r] = f32_round_down(s - E);
    }
  }
}

// one arrival per block on *ctr after an agent-scope release; true in the block that arrives last,
// which then holds an agent-scope acquire of every other block's stores and resets the counter
typedef __attribute__((address_space(1))) unsigned gu32;
__device__ __forceinline__ bool last_block_arrival(unsigned* ctr_flat) {
  __shared__ int s_last;
  gu32* ctr = (gu32*)ctr_flat;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // every wave: its stores before the arrival
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // drops this CU's stale lines before the loads
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

template <typename TQ, typename TG>
__global__ __launch_bounds__(256) void eval_prep_kernel(EvalSide q, EvalSide g, EvalCommon c) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < c.nb; t += (int64_t)gridDim.x * 256) c.bucket[t] = 0;
  if (row < q.n_pad)
    prep_row<TQ, TG>(q, g, c, row, lane);
  else if (row < q.n_pad + g.n_pad)
    prep_row<TG, TQ>(g, q, c, row - q.n_pad, lane);
  if (!last_block_arrival(c.done)) return;
  __shared__ float red[12], qmax[3], gmax[3];
  block_err_max(q, red, qmax);
  block_err_max(g, red, gmax);
  const int slot = mode_slot(c.mode);
  if (q.off) side_thresholds(q, gmax[slot], c);
  if (g.off) side_thresholds(g, qmax[slot], c);
}

// ranks of one direction + (#rank<=1, <=5, <=10, sum of ranks) into st[0..4)
__device__ __forceinline__ void side_ranks(const EvalSide& A, int64_t n_m, int64_t* st,
                                           unsigned long long* red /* LDS [4][4] */) {
  unsigned long long r1 = 0, r5 = 0, r10 = 0, sum = 0;
  for (int64_t i = threadIdx.x; i < A.n; i += 256) {
    const int64_t r = gt_rank_of(A.cnt[i], A.sgt[i], n_m);
    A.ranks[i] = r;
    r1 += (r <= 1);
    r5 += (r <= 5);
    r10 += (r <= 10);
    sum += (unsigned long long)r;
  }
  for (int o = 32; o >= 1; o >>= 1) {
    r1 += __shfl_xor(r1, o, 64);
    r5 += __shfl_xor(r5, o, 64);
    r10 += __shfl_xor(r10, o, 64);
    sum += __shfl_xor(sum, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w] = r1;
    red[4 + w] = r5;
    red[8 + w] = r10;
    red[12 + w] = sum;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const unsigned long long* r = red + 4 * threadIdx.x;
    st[threadIdx.x] = (int64_t)(r[0] + r[1] + r[2] + r[3]);
  }
  __syncthreads();
}

template <typename TQ, typename TG>
__global__ __launch_bounds__(256) void eval_fix_kernel(EvalSide q, EvalSide g, EvalCommon c) {
  fixup_walk<TQ, TG>((const TQ*)q.raw, q.ld, q.inv, (const TG*)g.raw, g.ld, g.inv, c.d, q.off ? q.sgt : nullptr,
                     g.off ? g.sgt : nullptr, q.cnt, g.cnt, c.cand, c.nb, c.cap_b);
  if (!last_block_arrival(c.done + 1)) return;
  __shared__ unsigned long long red[16];
  // pair total, or the buffer size a retry needs if a bucket outgrew cap_b (cand_finalize_kernel)
  unsigned long long tot = 0, mx = 0;
  for (int64_t b = threadIdx.x; b < c.nb; b += 256) {
    const unsigned long long v = c.bucket[b];
    tot += v;
    mx = v > mx ? v : mx;
  }
  for (int o = 32; o >= 1; o >>= 1) {
    tot += __shfl_xor(tot, o, 64);
    const unsigned long long m2 = __shfl_xor(mx, o, 64);
    mx = m2 > mx ? m2 : mx;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w] = tot;
    red[4 + w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    tot = red[0] + red[1] + red[2] + red[3];
    mx = max(max(red[4], red[5]), max(red[6], red[7]));
    c.stats[8] = (int64_t)tot;
    c.stats[9] = (int64_t)mx > c.cap_b ? ((int64_t)mx + 1) * c.nb + c.nb + 1 : 0;
  }
  __syncthreads();
  if (q.off) side_ranks(q, g.n, c.stats, red);
  if (g.off) side_ranks(g, q.n, c.stats + 4, red);
}

template <typename TQ, typename TG>
static int launch_eval_typed(const EvalSide& q, const EvalSide& g, const EvalCommon& c, int phase, hipStream_t s) {
  if (phase == 0) {
    const unsigned blocks = (unsigned)((q.n_pad + g.n_pad + 3) / 4);
    hipLaunchKernelGGL((eval_prep_kernel<TQ, TG>), dim3(blocks), dim3(256), 0, s, q, g, c);
    return check_launch("eval_prep_kernel");
  }
  // 32 blocks per XCD: the last-arrival counter sees 256 atomics (the rank fix-up's 1024-block grid
  // is sized for millions of pairs; an evaluation of this kind holds thousands)
  hipLaunchKernelGGL((eval_fix_kernel<TQ, TG>), dim3(8u * 32u), dim3(256), 0, s, q, g, c);
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
