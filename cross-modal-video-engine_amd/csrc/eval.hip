// K14: one exact two-direction GT-rank evaluation of a resident problem in four launches
// (cmve_eval_ranks, host side in sim.hip):
//   1. eval_prep_kernel    K1 pack of BOTH sets, the exact fp64 GT score of every row of both
//                          directions (K5a) and zeroed counters: one wave per row, 4 rows per block
//                          (every CU busy), no tail; per-block err maxima into 16 atomic-max shards
//   2. sim_kernel<RANK>    K4 rank GEMM (certain counts + undecided pairs); each block folds the other
//                          set's err_max from the shards (scalar loads) and derives its rows' / columns'
//                          thresholds from the GT scores itself (SimArgs::thr_gt)
//   3. eval_fix_kernel     K5b fp64 re-score of the undecided pairs, 4 waves per block, no tail
//   4. eval_finish_kernel  a block per 256 rows: the 1-based ranks, R@1/5/10 + rank sums per direction
//                          (block sums added into the stats head); two more blocks: the pair total and
//                          overflow size, and the sets' err_max (from the prep's shards)
// Round 2 first ran this as three launches whose LAST blocks derived the thresholds and the ranks
// (an agent-scope arrival hand-off): per-block stamps put ~5-6 us on each arrival chain and 4-7 us on
// each one-block tail, against ~1 us per kernel boundary; the boundaries replace them.
// It replaces the per-evaluation chain of the reference's validation / test loop
// (LINAS-engine/validate.py:61-74, tester.py:133-139): evaluation.cal_error (evaluation.py:17-21,
// both sets re-normalised, the full matrix in fp64) -> util/metrics.eval_q2m in both directions
// (metrics.py:124-157, an argsort per row).  The separate-launch path (cmve_pack_rows x2,
// cmve_gt_thresholds x2, cmve_rank_count, cmve_gt_ranks x2) computes the identical numbers: the
// pack, GT-score and fix-up arithmetic are the same device functions (cmve_internal.h).
#include "eval_abi.h"

namespace cmve {

// The register-resident pieces of the prep for rows of <= 1024 elements that both sides read in 16-B
// pieces (rows_vec4): a row is loaded ONCE into registers (16 doubles per lane, elements 4L + 256m + c)
// and normalised, packed and dotted from there.  Every per-lane accumulation runs in the (m, c) order of
// row_sumsq / pack_row_planes / wave_dot64, so the planes, bounds, norms and GT scores are bit-identical
// to the streaming path (and to cmve_pack_rows / cmve_gt_thresholds).
template <typename T>
__device__ __forceinline__ void load_row_regs(const T* __restrict__ x, int64_t d, int lane, double (&v)[4][4]) {
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int64_t k = (int64_t)lane * 4 + 256 * m;
    if (k < d) load4d(x + k, v[m]);
    else v[m][0] = v[m][1] = v[m][2] = v[m][3] = 0.0;
  }
}

// this lane's fma chains (before the wave sum): sum of squares / dot product in (m, c) order
__device__ __forceinline__ double lane_sumsq(const double (&v)[4][4], int64_t d, int lane) {
  double ss = 0.0;
#pragma unroll
  for (int m = 0; m < 4; ++m)
    if ((int64_t)lane * 4 + 256 * m < d)
#pragma unroll
      for (int q = 0; q < 4; ++q) ss = fma(v[m][q], v[m][q], ss);
  return ss;
}
__device__ __forceinline__ double lane_dot(const double (&v)[4][4], const double (&w)[4][4], int64_t d, int lane) {
  double dot = 0.0;
#pragma unroll
  for (int m = 0; m < 4; ++m)
    if ((int64_t)lane * 4 + 256 * m < d)
#pragma unroll
      for (int q = 0; q < 4; ++q) dot = fma(v[m][q], w[m][q], dot);
  return dot;
}

// the wave sums of K independent values in ONE butterfly (wave_sum's pairings and order for each: the same
// bits as K wave_sum calls, one reduction latency instead of K)
template <int K>
__device__ __forceinline__ void wave_sum_k(double (&v)[K]) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += __shfl_xor(v[k], o, 64);
}

// pack row `row` of side A (held in v) into its planes with 1/||x|| = inv, accumulating this lane's squared
// residuals in acc (not yet reduced); pack_bounds stores inv and the bounds from the reduced sums
__device__ __forceinline__ void pack_regs_lane(const EvalSide& A, const EvalCommon& c, int64_t row,
                                               const double (&v)[4][4], double inv, int lane, PackAcc& acc);
__device__ __forceinline__ bool pack_bf(const EvalSide& A, const EvalCommon& c) {
  return !(c.mode == CMVE_SIM_F16 && A.h16 != nullptr);
}
__device__ __forceinline__ void pack_bounds(const EvalSide& A, int64_t row, double inv, bool bf, double e1, double e2,
                                            double e3, int lane, float (&eb)[3], double e4 = 0.0) {
  if (lane == 0) {
    gst(A.inv + row, inv);
    if (A.lo16) A.err_lo16[row] = lo16_bound(e4);  // (lo16_elem's residuals)
    // pack_row_planes' bounds
    eb[0] = bf ? f32_round_up(sqrt(e1) * (1.0 + 1e-9) + 1e-12) : INFINITY;
    eb[1] = bf ? f32_round_up(sqrt(e2) * (1.0 + 1e-9) + 1e-12) : INFINITY;
    eb[2] = A.err_h16 ? f32_round_up(sqrt(e3) * (1.0 + 1e-9) + 1e-12) : 0.f;
    gst(A.err_hi + row, eb[0]);
    gst(A.err_hilo + row, eb[1]);
    if (A.err_h16) gst(A.err_h16 + row, eb[2]);
  }
}

// pack row `row` of side A (held in v) into its planes with 1/||x|| = inv; lane 0 stores inv and the
// bounds; eb = the row's bounds (lane 0)
__device__ __forceinline__ void pack_regs(const EvalSide& A, const EvalCommon& c, int64_t row,
                                          const double (&v)[4][4], double inv, int lane, float (&eb)[3]) {
  PackAcc acc;
  pack_regs_lane(A, c, row, v, inv, lane, acc);
  const bool bf = pack_bf(A, c);
  const double e1 = bf ? wave_sum(acc.e1) : 0.0, e2 = bf ? wave_sum(acc.e2) : 0.0, e3 = wave_sum(acc.e3);
  const double e4 = A.lo16 ? wave_sum((double)acc.e4) : 0.0;
  pack_bounds(A, row, inv, bf, e1, e2, e3, lane, eb, e4);
}

__device__ __forceinline__ void pack_regs_lane(const EvalSide& A, const EvalCommon& c, int64_t row,
                                               const double (&v)[4][4], double inv, int lane, PackAcc& acc) {
  uint16_t* hrow = A.hi + row * c.d_pad;
  uint16_t* lrow = A.lo ? A.lo + row * c.d_pad : nullptr;
  uint16_t* frow = A.h16 ? A.h16 + row * c.d_pad : nullptr;
  const bool want_f16 = frow != nullptr;
  if (c.mode == CMVE_SIM_F16 && want_f16) {
    // the F16 rank GEMM reads only the fp16 plane: the bf16 planes are not written and their bounds
    // are +inf (a stale plane can never pass for a bounded one); with A.lo16 the bf16 residual plane of the
    // level-2 re-score is written beside it (lo16_elem: two fp32 ops and a conversion per element)
    uint16_t* lrow16 = A.lo16 ? A.lo16 + row * c.d_pad : nullptr;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int64_t k = (int64_t)lane * 4 + 256 * m;
      if (k >= c.d_pad) break;
      cmve_u16x4 fv = {0, 0, 0, 0}, lv = {0, 0, 0, 0};
      if (k < c.d) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const double xh = v[m][q] * inv;
          float xf;
          const _Float16 hf16 = f16_via_f32(xh, xf);  // pack_elem's f16 arithmetic
          const double r3 = xh - (double)hf16;
          acc.e3 = fma(r3, r3, acc.e3);
          fv[q] = __builtin_bit_cast(uint16_t, hf16);
          if (lrow16) {
            float res;
            lv[q] = lo16_elem(xf, hf16, res);
            acc.e4 = fmaf(res, res, acc.e4);
          }
        }
      }
      gst((cmve_u16x4*)(frow + k), fv);
      if (lrow16) gst((cmve_u16x4*)(lrow16 + k), lv);
      asm volatile("" : "+v"(acc.e3), "+v"(acc.e4));  // (pack_f16_lo16: the chunk's sums complete here)
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
      gst((cmve_u16x4*)(hrow + k), hv);
      if (lrow) gst((cmve_u16x4*)(lrow + k), lv);
      if (frow) gst((cmve_u16x4*)(frow + k), fv);
    }
  }
}

template <typename TA, typename TB>
__device__ __forceinline__ void prep_row_regs(const EvalSide& A, const EvalSide& B, const EvalCommon& c, int64_t row,
                                              const TA* __restrict__ x, int lane, float (&eb)[3]) {
  // the first GT partner's row is loaded beside the row itself (its index is known up front): the
  // GT score then needs no second HBM round trip after the pack
  const int64_t g_beg = A.off ? gld(A.off + row) : 0, g_end = A.off ? gld(A.off + row + 1) : 0;
  double w0[4][4];
  if (g_beg < g_end) load_row_regs((const TB*)B.raw + (int64_t)gld(A.idx + g_beg) * B.ld, c.d, lane, w0);
  double v[4][4];
  load_row_regs(x, c.d, lane, v);
  const double inv = row_inv_norm(wave_sum(lane_sumsq(v, c.d, lane)), A.eps, A.flags);
  pack_regs(A, c, row, v, inv, lane, eb);
  if (!A.off) return;
  double best = -INFINITY;
  bool any = false;
  for (int64_t g = g_beg; g < g_end; ++g) {
    double w[4][4];
    if (g == g_beg) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int q = 0; q < 4; ++q) w[m][q] = w0[m][q];
    } else {
      load_row_regs((const TB*)B.raw + (int64_t)gld(A.idx + g) * B.ld, c.d, lane, w);
    }
    const double invb = row_inv_norm(wave_sum(lane_sumsq(w, c.d, lane)), B.eps, B.flags);
    const double s = wave_sum(lane_dot(v, w, c.d, lane)) * (inv * invb);  // wave_cos64(x, y, inv, invb)
    if (s == s) {
      any = true;
      if (s > best) best = s;
    }
  }
  if (lane == 0) {
    gst(A.sgt + row, any ? best : (g_end > g_beg ? (double)INFINITY : (double)NAN));
    gst(A.cnt + row, 0);
    if (A.gt1) gst(A.gt1 + row, g_end > g_beg ? gld(A.idx + g_beg) : -1);
  }
}

// pack row `row` of side A and score its GT list against side B (one wave)
template <typename TA, typename TB>
__device__ __forceinline__ void prep_row(const EvalSide& A, const EvalSide& B, const EvalCommon& c, int64_t row,
                                         int lane, float (&eb)[3]) {
  uint16_t* hrow = A.hi + row * c.d_pad;
  uint16_t* lrow = A.lo ? A.lo + row * c.d_pad : nullptr;
  uint16_t* frow = A.h16 ? A.h16 + row * c.d_pad : nullptr;
  if (row >= A.n) {  // padding rows: zero vectors, zero bounds, never counted
    pack_pad_row(hrow, lrow, frow, c.d_pad, lane);
    if (lane == 0) {
      gst(A.inv + row, 0.0);
      gst(A.err_hi + row, 0.f);
      gst(A.err_hilo + row, 0.f);
      if (A.err_h16) gst(A.err_h16 + row, 0.f);
      if (A.off) {
        gst(A.sgt + row, (double)NAN);
        gst(A.cnt + row, 0);
        if (A.gt1) gst(A.gt1 + row, -1);
      }
    }
    return;
  }
  const TA* x = (const TA*)A.raw + row * A.ld;
  if (A.vec && B.vec && c.d_pad <= 1024) {
    prep_row_regs<TA, TB>(A, B, c, row, x, lane, eb);
    return;
  }
  const double inv = row_inv_norm(row_sumsq<TA>(x, c.d, A.vec != 0, lane), A.eps, A.flags);
  float b1, b2, b3;
  pack_row_planes<TA>(x, c.d, c.d_pad, A.vec != 0, inv, hrow, lrow, frow, lane, b1, b2, b3);
  if (lane == 0) {
    gst(A.inv + row, inv);
    gst(A.err_hi + row, eb[0] = b1);
    gst(A.err_hilo + row, eb[1] = b2);
    eb[2] = A.err_h16 ? b3 : 0.f;
    if (A.err_h16) gst(A.err_h16 + row, b3);
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
    gst(A.sgt + row, any ? best : (A.off[row + 1] > A.off[row] ? (double)INFINITY : (double)NAN));
    gst(A.cnt + row, 0);
    if (A.gt1) gst(A.gt1 + row, A.off[row + 1] > A.off[row] ? A.idx[A.off[row]] : -1);
  }
}

constexpr int FIN_NT = 256;  // finish: 256 rows per block, one block per 256 rows of the larger side
constexpr int FIN_NW = FIN_NT / 64;

// reduce K values per thread over a block of FIN_NT threads in ONE LDS round (max or sum); every
// thread gets the K results in v
template <bool MAX, typename T, int K>
__device__ __forceinline__ void block_reduce_k(T (&v)[K], T* red /* LDS [K + 1][FIN_NW] */) {
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const T u = __shfl_xor(v[k], o, 64);
      v[k] = MAX ? (u > v[k] ? u : v[k]) : v[k] + u;
    }
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) red[k * FIN_NW + (threadIdx.x >> 6)] = v[k];
  __syncthreads();
  T* out = red + K * FIN_NW;  // thread k < K folds row k (wave order: deterministic)
  if (threadIdx.x < K) {
    const T* r = red + threadIdx.x * FIN_NW;
    T a = r[0];
#pragma unroll
    for (int w = 1; w < FIN_NW; ++w) a = MAX ? (r[w] > a ? r[w] : a) : a + r[w];
    out[threadIdx.x] = a;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = out[k];
}

#ifndef CMVE_PREP_NT
#define CMVE_PREP_NT 256
#endif
constexpr int PREP_NT = CMVE_PREP_NT;  // 4 rows per block: a 1k-A evaluation's 2,048 rows fill every CU
constexpr int PREP_NW = PREP_NT / 64;

template <typename TQ, typename TG>
__device__ __forceinline__ void eval_prep_body(const EvalSide& q, const EvalSide& g, const EvalCommon& c) {
  EVAL_STAMP(c, 0, 0);
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * PREP_NW + (threadIdx.x >> 6);
  for (int64_t t = (int64_t)blockIdx.x * PREP_NT + threadIdx.x; t < c.nb; t += (int64_t)gridDim.x * PREP_NT)
    gst(c.bucket + t, 0ull);
  if (blockIdx.x == 0 && threadIdx.x < 13) gst(c.stats + threadIdx.x, 0);  // the finish blocks add into it
  if (blockIdx.x == 0 && threadIdx.x == 0 && c.l3_count) gst(c.l3_count, 0u);  // the rank GEMM appends level 3
  float eb[3] = {0.f, 0.f, 0.f};  // this wave's row bounds (lane 0; padding rows 0)
  if (!(c.dbg & 1)) {
    if (row < q.n_pad)
      prep_row<TQ, TG>(q, g, c, row, lane, eb);
    else if (row < q.n_pad + g.n_pad)
      prep_row<TG, TQ>(g, q, c, row - q.n_pad, lane, eb);
  }
  // err_max shards: the block's max per plane (its 4 rows are one side: n_pad % 4 == 0), one atomic
  // max on the float bits per plane into shard blockIdx % EMAX_SHARDS of its side (bounds are >= 0 or
  // +inf; NaN dropped by fmaxf); 64 shards keep ~8 same-address atomics per shard for a 1k-A prep
  // (16 shards: ~3 us of serialised atomics at the end of the launch).  The rank GEMM folds the shards of the mode's plane, the finish folds
  // all of them into the sets' err_max and zeroes them for the next evaluation.
  __shared__ float s_eb[PREP_NW][3];
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 3; ++k) s_eb[threadIdx.x >> 6][k] = eb[k];
  __syncthreads();
  if (threadIdx.x < 3) {
    float m = 0.f;
#pragma unroll
    for (int w = 0; w < PREP_NW; ++w) m = fmaxf(m, s_eb[w][threadIdx.x]);
    const int side = (int64_t)blockIdx.x * PREP_NW < q.n_pad ? 0 : 1;
    unsigned* sh = &c.emax[(side * 3 + threadIdx.x) * EMAX_SHARDS + blockIdx.x % EMAX_SHARDS];
    // +inf (a plane the mode does not write) is the largest value: a plain store equals the atomic max
    if (c.dbg & 2) {  // kernel studies only: no err_max shards (results garbage)
    } else if (m == INFINITY) gst(sh, __float_as_uint(m));
    else if (m > 0.f) gmax(sh, __float_as_uint(m));
  }
  EVAL_STAMP(c, 0, 1);
}

// The prep of a one-to-one GT pairing (cmve_eval_ranks with CMVE_EVAL_PAIRED: caption i's only GT is
// video p = q.idx[q.off[i]] and video p's only GT is caption i -- MSR-VTT-1kA's structure): ONE wave per
// (caption, video) pair loads both rows once, packs both and scores the pair once for both directions.
// Half the waves and half the row reads of eval_prep_kernel (which loads every row twice: as a row and as
// its partner's GT), and the same bits: each side's norm, planes and bounds come from the same register
// code, and the GT score fma(v, w) chain is symmetric in the two rows.  Padding rows i >= n of both sides
// are this wave's too (q.n == g.n, q.n_pad == g.n_pad).
template <typename TQ, typename TG>
__device__ __forceinline__ void eval_prep_pair_body(const EvalSide& q, const EvalSide& g, const EvalCommon& c) {
  EVAL_STAMP(c, 0, 0);
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * PREP_NW + (threadIdx.x >> 6);
  for (int64_t t = (int64_t)blockIdx.x * PREP_NT + threadIdx.x; t < c.nb; t += (int64_t)gridDim.x * PREP_NT)
    gst(c.bucket + t, 0ull);
  if (blockIdx.x == 0 && threadIdx.x < 13) gst(c.stats + threadIdx.x, 0);  // the finish blocks add into it
  if (blockIdx.x == 0 && threadIdx.x == 0 && c.l3_count) gst(c.l3_count, 0u);  // the rank GEMM appends level 3
  float ebq[3] = {0.f, 0.f, 0.f}, ebg[3] = {0.f, 0.f, 0.f};
  if (i < q.n_pad && !(c.dbg & 1)) {
    if (i >= q.n) {  // padding rows of both sides: zero vectors, zero bounds, never counted
      const EvalSide* sides[2] = {&q, &g};
#pragma unroll
      for (int sd = 0; sd < 2; ++sd) {
        const EvalSide& A = *sides[sd];
        pack_pad_row(A.hi + i * c.d_pad, A.lo ? A.lo + i * c.d_pad : nullptr, A.h16 ? A.h16 + i * c.d_pad : nullptr,
                     c.d_pad, lane);
        if (lane == 0) {
          gst(A.inv + i, 0.0);
          gst(A.err_hi + i, 0.f);
          gst(A.err_hilo + i, 0.f);
          if (A.err_h16) gst(A.err_h16 + i, 0.f);
          gst(A.sgt + i, (double)NAN);
          gst(A.cnt + i, 0);
          if (A.gt1) gst(A.gt1 + i, -1);
        }
      }
    } else {
      // the caller asserts a one-to-one pairing; its t2v side is checked here (one GT per caption, a real video)
      // so that lists which are not one never write out of range: such a row writes nothing of side g, gets an
      // empty GT list (q.sgt NaN) and gt1 = -2, which the finish counts into stats[11] (the host mirror raises
      // on it).  (Two captions naming one video -- lists that are not a bijection -- give undefined ranks, as the
      // contract says, but every write stays inside that video's row.)
      const int64_t qb = gld(q.off + i);
      const int64_t p0 = gld(q.off + i + 1) - qb == 1 ? (int64_t)gld(q.idx + qb) : -1;
      const bool valid = p0 >= 0 && p0 < g.n;
      const int64_t p = valid ? p0 : 0;  // (row 0 is a real row: loaded, never written when invalid)
      double v[4][4], w[4][4];
      load_row_regs((const TQ*)q.raw + i * q.ld, c.d, lane, v);
      load_row_regs((const TG*)g.raw + p * g.ld, c.d, lane, w);
      if (!valid) {
        double e[1] = {lane_sumsq(v, c.d, lane)};
        wave_sum_k<1>(e);
        const double invq = row_inv_norm(e[0], q.eps, q.flags);
        pack_regs(q, c, i, v, invq, lane, ebq);
        if (lane == 0) {
          gst(q.sgt + i, (double)NAN);
          gst(q.cnt + i, 0);
          if (q.gt1) gst(q.gt1 + i, -2);
        }
      } else {
      // both norms and the pair's dot in one butterfly, then both planes' residual sums in another (each sum
      // in wave_sum's order: the bits of the separate reductions)
      double r3[3] = {lane_sumsq(v, c.d, lane), lane_sumsq(w, c.d, lane), lane_dot(v, w, c.d, lane)};
      wave_sum_k<3>(r3);
      const double invq = row_inv_norm(r3[0], q.eps, q.flags), invg = row_inv_norm(r3[1], g.eps, g.flags);
      PackAcc aq, ag;
      pack_regs_lane(q, c, i, v, invq, lane, aq);
      pack_regs_lane(g, c, p, w, invg, lane, ag);
      const bool bfq = pack_bf(q, c), bfg = pack_bf(g, c);
      if (!bfq && !bfg) {  // the F16 rank GEMM's planes: only the fp16 (and r8) residuals
        double e[4] = {aq.e3, ag.e3, (double)aq.e4, (double)ag.e4};
        wave_sum_k<4>(e);
        pack_bounds(q, i, invq, false, 0.0, 0.0, e[0], lane, ebq, e[2]);
        pack_bounds(g, p, invg, false, 0.0, 0.0, e[1], lane, ebg, e[3]);
      } else {
        double e[6] = {aq.e1, aq.e2, aq.e3, ag.e1, ag.e2, ag.e3};
        wave_sum_k<6>(e);
        pack_bounds(q, i, invq, bfq, bfq ? e[0] : 0.0, bfq ? e[1] : 0.0, e[2], lane, ebq);
        pack_bounds(g, p, invg, bfg, bfg ? e[3] : 0.0, bfg ? e[4] : 0.0, e[5], lane, ebg);
      }
      const double s = r3[2] * (invq * invg);
      if (lane == 0) {  // a one-entry list: its score, or +inf when it is NaN (prep_row_regs' encoding)
        gst(q.sgt + i, s == s ? s : (double)INFINITY);
        gst(g.sgt + p, s == s ? s : (double)INFINITY);
        gst(q.cnt + i, 0);
        gst(g.cnt + p, 0);
        if (q.gt1) gst(q.gt1 + i, (int32_t)p);
        if (g.gt1) gst(g.gt1 + p, (int32_t)i);
      }
      }
    }
  }
  // err_max shards of both sides (eval_prep_kernel's scheme)
  __shared__ float s_eb[PREP_NW][6];
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      s_eb[threadIdx.x >> 6][k] = ebq[k];
      s_eb[threadIdx.x >> 6][3 + k] = ebg[k];
    }
  __syncthreads();
  if (threadIdx.x < 6) {
    float m = 0.f;
#pragma unroll
    for (int w = 0; w < PREP_NW; ++w) m = fmaxf(m, s_eb[w][threadIdx.x]);
    unsigned* sh = &c.emax[threadIdx.x * EMAX_SHARDS + blockIdx.x % EMAX_SHARDS];  // [side][plane] = tid
    if (c.dbg & 2) {  // kernel studies only: no err_max shards (results garbage)
    } else if (m == INFINITY) gst(sh, __float_as_uint(m));
    else if (m > 0.f) gmax(sh, __float_as_uint(m));
  }
  EVAL_STAMP(c, 0, 1);
}

// The paired prep of the F16 rank path with the level-2 plane (the 1k-A headline's form): rows of exactly
// d = d_pad = 256 NM elements, read in 16-B pieces (rows_vec4), so no element guards.  The same arithmetic as
// eval_prep_pair_body -- the norms, the GT dot, the fp16 plane and its bound in the same (m, c) fma order, so
// h16 / inv_norm / err_h16 / the GT scores are bit-identical to it -- with the bf16 residual plane
// (lo16_elem: the hardware bf16 conversion, fp32 residuals) written beside the fp16 plane.
template <int NM>
__device__ __forceinline__ void pack_f16_lo16(const EvalSide& A, int64_t row, const double (&v)[NM][4], double inv,
                                              int lane, bool store, double& e3, float& e4) {
  // The planes are stored WRITE-THROUGH (sc1): their lines leave the XCD's L2 clean, so this launch's end-of-kernel
  // release (buffer_wbl2) has ~8 MB per evaluation less to write back before the rank GEMM may start
  // (MI355X_MICROARCH.md, visibility: a release costs ~1.7 us clean, several us freshly dirtied; the eval stamps
  // measured a 5.3 us gap between the last prep block and the first rank-GEMM block).  16-B sc1 stores cost what
  // plain ones do, narrower ones several times more, so lanes L and L ^ 1 swap halves of two chunks (one DPP swap
  // per dword) and each stores 16 contiguous bytes: the even lane chunk m's [4L, 4L + 8), the odd lane chunk m + 1's
  // [4L - 4, 4L + 4).
  uint16_t* frow = A.h16 + row * (int64_t)(NM * 256);
  uint16_t* lrow = A.lo16 + row * (int64_t)(NM * 256);
  const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc((void*)frow, 0, NM * 512, 0x00020000);
  const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc((void*)lrow, 0, NM * 512, 0x00020000);
  const bool odd = lane & 1;
  cmve_u32x2 pf = {0u, 0u}, pl = {0u, 0u};  // an even chunk's values, held for its pair
  auto swap = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false); };
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    cmve_u16x4 fv, lv;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const double xh = v[m][q] * inv;
      float xf;
      const _Float16 h = f16_via_f32(xh, xf);  // pack_elem's f16 arithmetic
      const float hf = (float)h;
      const double r3 = xh - (double)hf;
      e3 = fma(r3, r3, e3);
      const float d2 = xf - hf;
      const __bf16 lo = (__bf16)d2;
      const float res = d2 - (float)lo;
      e4 = fmaf(res, res, e4);
      fv[q] = __builtin_bit_cast(uint16_t, h);
      lv[q] = __builtin_bit_cast(uint16_t, lo);
    }
    const cmve_u32x2 f2 = __builtin_bit_cast(cmve_u32x2, fv), l2 = __builtin_bit_cast(cmve_u32x2, lv);
    if (store) {
      if ((m & 1) == 0 && m + 1 < NM) {
        pf = f2;
        pl = l2;
      } else if (m & 1) {
        const cmve_u32x2 sf = odd ? pf : f2, sl = odd ? pl : l2;  // what the partner lane needs
        const cmve_u32x2 rf2 = {swap(sf.x), swap(sf.y)}, rl2 = {swap(sl.x), swap(sl.y)};
        const cmve_u32x4 df = odd ? cmve_u32x4{rf2.x, rf2.y, f2.x, f2.y} : cmve_u32x4{pf.x, pf.y, rf2.x, rf2.y};
        const cmve_u32x4 dl = odd ? cmve_u32x4{rl2.x, rl2.y, l2.x, l2.y} : cmve_u32x4{pl.x, pl.y, rl2.x, rl2.y};
        const int off = odd ? (m * 256 + 4 * (lane - 1)) * 2 : ((m - 1) * 256 + 4 * lane) * 2;
        __builtin_amdgcn_raw_buffer_store_b128(df, rf, off, 0, 16);  // (aux 16: sc1)
        __builtin_amdgcn_raw_buffer_store_b128(dl, rl, off, 0, 16);
      } else {  // the last chunk of an odd NM: 8 B per lane
        __builtin_amdgcn_raw_buffer_store_b64(f2, rf, (m * 256 + 4 * lane) * 2, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b64(l2, rl, (m * 256 + 4 * lane) * 2, 0, 16);
      }
    }
    // the chunk's residual sums complete here (left free, the compiler sank every fma chain below the last
    // chunk's stores and held all 32 elements' temporaries: ~190 registers)
    asm volatile("" : "+v"(e3), "+v"(e4));
  }
}

// a raw row of d = 256 NM elements into registers (lane L: elements 4L + 256m + c) through a buffer resource:
// one VGPR offset for every load of the row, the 256-element steps in scalar offsets (per-load 64-bit
// addresses held ~64 registers and pushed the prep past 128)
typedef uint32_t prep_u32x4 __attribute__((ext_vector_type(4)));
#ifndef CMVE_PREP_ROW_AUX
#define CMVE_PREP_ROW_AUX 0  // the raw rows' cache policy (gfx950 buffer aux bits: 2 = nt, 1 = sc0, 16 = sc1)
#endif
typedef double prep_f64x2 __attribute__((ext_vector_type(2)));
template <int NM>
__device__ __forceinline__ void load_row_buf(const double* row, int lane, double (&v)[NM][4]) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)row, 0, NM * 256 * 8, 0x00020000);
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    const prep_f64x2 a = __builtin_bit_cast(prep_f64x2, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 32, m * 2048, CMVE_PREP_ROW_AUX));
    const prep_f64x2 b =
        __builtin_bit_cast(prep_f64x2, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 32 + 16, m * 2048, CMVE_PREP_ROW_AUX));
    v[m][0] = a.x;
    v[m][1] = a.y;
    v[m][2] = b.x;
    v[m][3] = b.y;
  }
}
template <int NM>
__device__ __forceinline__ void load_row_buf(const float* row, int lane, double (&v)[NM][4]) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)row, 0, NM * 256 * 4, 0x00020000);
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    const cmve_f32x4 a = __builtin_bit_cast(cmve_f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, m * 1024, CMVE_PREP_ROW_AUX));
    v[m][0] = a.x;
    v[m][1] = a.y;
    v[m][2] = a.z;
    v[m][3] = a.w;
  }
}

template <typename TQ, typename TG, int NM>
__device__ __forceinline__ void eval_prep_pair_f16_body(const EvalSide& q, const EvalSide& g, const EvalCommon& c,
                                                        int64_t vb, int64_t nvb) {
  // vb / nvb: this block and the prep's block count (blockIdx.x / gridDim.x, or the prep blocks' own numbering in
  // eval_prep_fin_batch_kernel)
  EVAL_STAMP(c, 0, 0);
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)vb * PREP_NW + (threadIdx.x >> 6);
  for (int64_t t = (int64_t)vb * PREP_NT + threadIdx.x; t < c.nb; t += (int64_t)nvb * PREP_NT)
    gst(c.bucket + t, 0ull);
  if (vb == 0 && threadIdx.x < 13) gst(c.stats + threadIdx.x, 0);  // the finish blocks add into it
  if (vb == 0 && threadIdx.x == 0 && c.l3_count) gst(c.l3_count, 0u);  // the rank GEMM appends level 3
  float ebq[3] = {0.f, 0.f, 0.f}, ebg[3] = {0.f, 0.f, 0.f};
  if (i < q.n_pad && !(c.dbg & 1)) {
    if (i >= q.n) {  // padding rows of both sides: zero vectors, zero bounds, never counted
      const EvalSide* sides[2] = {&q, &g};
#pragma unroll
      for (int sd = 0; sd < 2; ++sd) {
        const EvalSide& A = *sides[sd];
        pack_pad_row(A.hi + i * c.d_pad, A.lo ? A.lo + i * c.d_pad : nullptr, A.h16 + i * c.d_pad, c.d_pad, lane);
        if (lane == 0) {
          gst(A.inv + i, 0.0);
          gst(A.err_hi + i, 0.f);
          gst(A.err_hilo + i, 0.f);
          gst(A.err_h16 + i, 0.f);
          gst(A.sgt + i, (double)NAN);
          gst(A.cnt + i, 0);
          if (A.gt1) gst(A.gt1 + i, -1);
        }
      }
    } else {
      // (eval_prep_pair_body's check of the t2v side of the pairing)
      const int64_t qb = gld(q.off + i);
      const int64_t p0 = gld(q.off + i + 1) - qb == 1 ? (int64_t)gld(q.idx + qb) : -1;
      const bool valid = p0 >= 0 && p0 < g.n;
      const int64_t p = valid ? p0 : 0;
      double v[NM][4], w[NM][4];
      load_row_buf<NM>((const TQ*)q.raw + i * q.ld, lane, v);
      load_row_buf<NM>((const TG*)g.raw + p * g.ld, lane, w);
      double r3[3] = {0.0, 0.0, 0.0};  // lane_sumsq(v), lane_sumsq(w), lane_dot(v, w): the same fma order
#pragma unroll
      for (int m = 0; m < NM; ++m)
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          r3[0] = fma(v[m][q4], v[m][q4], r3[0]);
          r3[1] = fma(w[m][q4], w[m][q4], r3[1]);
          r3[2] = fma(v[m][q4], w[m][q4], r3[2]);
        }
      wave_sum_k<3>(r3);
      const double invq = row_inv_norm(r3[0], q.eps, q.flags), invg = row_inv_norm(r3[1], g.eps, g.flags);
      double e3q = 0.0, e3g = 0.0;
      float e4q = 0.f, e4g = 0.f;
      // (one side after the other, one 4-element chunk at a time: left to itself the scheduler interleaves the
      // two sides' chunks and holds ~190 registers, which caps the prep at two waves per SIMD)
      pack_f16_lo16<NM>(q, i, v, invq, lane, true, e3q, e4q);
      __builtin_amdgcn_sched_barrier(0);
      pack_f16_lo16<NM>(g, p, w, invg, lane, valid, e3g, e4g);
      double e[4] = {e3q, e3g, (double)e4q, (double)e4g};
      wave_sum_k<4>(e);
      pack_bounds(q, i, invq, false, 0.0, 0.0, e[0], lane, ebq, e[2]);
      if (valid) pack_bounds(g, p, invg, false, 0.0, 0.0, e[1], lane, ebg, e[3]);
      const double sc = r3[2] * (invq * invg);
      if (lane == 0) {
        gst(q.sgt + i, !valid ? (double)NAN : (sc == sc ? sc : (double)INFINITY));
        gst(q.cnt + i, 0);
        if (q.gt1) gst(q.gt1 + i, valid ? (int32_t)p : -2);
        if (valid) {
          gst(g.sgt + p, sc == sc ? sc : (double)INFINITY);
          gst(g.cnt + p, 0);
          if (g.gt1) gst(g.gt1 + p, (int32_t)i);
        }
      }
    }
  }
  // err_max shards of both sides (eval_prep_kernel's scheme)
  __shared__ float s_eb[PREP_NW][6];
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      s_eb[threadIdx.x >> 6][k] = ebq[k];
      s_eb[threadIdx.x >> 6][3 + k] = ebg[k];
    }
  __syncthreads();
  if (threadIdx.x < 6) {
    float m = 0.f;
#pragma unroll
    for (int w = 0; w < PREP_NW; ++w) m = fmaxf(m, s_eb[w][threadIdx.x]);
    unsigned* sh = &c.emax[threadIdx.x * EMAX_SHARDS + vb % EMAX_SHARDS];  // [side][plane] = tid
    if (c.dbg & 2) {  // kernel studies only: no err_max shards (results garbage)
    } else if (m == INFINITY) gst(sh, __float_as_uint(m));
    else if (m > 0.f) gmax(sh, __float_as_uint(m));
  }
  EVAL_STAMP(c, 0, 1);
}

constexpr int FIX_NT = 256;
#ifndef CMVE_FIX_BLOCKS
#define CMVE_FIX_BLOCKS 1024
#endif
#ifndef CMVE_FIXB_BLOCKS
#define CMVE_FIXB_BLOCKS 192  // (x 4 waves x 2 pairs: ~1,600 listed pairs of a 1k-A evaluation in one step)
#endif

// the fix-up of an evaluation with the level-2 planes (d_pad <= 1024): one flat walk over the buckets, TWO listed
// pairs per wave per step with every level-2 load of both in flight (one round trip of 16 KiB), the directions
// whose GT score lies outside s2 +- E2 decided there, fp64 (wave_cos64) for the few left
// (vb, nvb: this block among the walk's blocks -- blockIdx.x / gridDim.x, or a role's own numbering in a shared
// launch; MAXB: the bucket capacity of the LDS prefix)
template <typename TQ, typename TG, int64_t MAXB = FIXUP_MAX_BUCKETS_PER_XCD>
__device__ __forceinline__ void eval_fix2_walk(const EvalSide& q, const EvalSide& g, const EvalCommon& c, int64_t vb,
                                               int64_t nvb) {
  __shared__ int64_t pre[MAXB + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t nb = c.nb, ldk = c.d_pad;
  if (wave == 0) fixup_prefix(c.cand, nb, c.cap_b, 0, 1, nb, lane, pre);
  __syncthreads();
  const int64_t total = pre[nb];
  const int nw = (int)(blockDim.x >> 6);
  const int64_t stride = nvb * nw * 2;
  int64_t kb = 0;
  auto entry = [&](int64_t cc) -> uint64_t {  // pair cc of the walk (0: none); cc increases call by call
    if (cc >= total) return 0ull;
    if (pre[kb + 1] <= cc) {
      int64_t lo = kb + 1, hi = nb - 1;
      while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= cc) lo = mid;
        else hi = mid - 1;
      }
      kb = lo;
    }
    return gld(c.cand + nb + kb * c.cap_b + (cc - pre[kb]));
  };
  const bool dq = q.off != nullptr, dg = g.off != nullptr;
  for (int64_t c0 = (vb * nw + wave) * 2; c0 < total; c0 += stride) {
    const uint64_t u[2] = {entry(c0), entry(c0 + 1)};
    int64_t pi[2], pj[2];
    uint32_t fl[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      pi[t] = (int64_t)(u[t] & 0x7fffffffull);
      pj[t] = (int64_t)((u[t] >> 31) & 0x7fffffffull);
      fl[t] = (uint32_t)(u[t] >> 62) & ((dq ? 1u : 0u) | (dg ? 2u : 0u));
    }
    double s2[2] = {0.0, 0.0};
    const int64_t k = 16 * (int64_t)lane;
    if (k < ldk) {
      L16Frag fa[2], fb[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        l16_load(q.h16 + pi[t] * ldk, q.lo16 + pi[t] * ldk, k, fa[t]);  // (a null entry reads row 0: harmless)
        l16_load(g.h16 + pj[t] * ldk, g.lo16 + pj[t] * ldk, k, fb[t]);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) s2[t] = l16_partial(fa[t], fb[t], 0.0);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      s2[0] += __shfl_xor(s2[0], o, 64);
      s2[1] += __shfl_xor(s2[1], o, 64);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (!fl[t]) continue;  // (wave-uniform)
      const double eq = (double)gld(q.err_lo16 + pi[t]), eg = (double)gld(g.err_lo16 + pj[t]);
      const double E2 = eq + (1.0 + eq) * eg + 2e-12;
      const double tq = (fl[t] & 1u) ? gld(q.sgt + pi[t]) : 0.0, tg = (fl[t] & 2u) ? gld(g.sgt + pj[t]) : 0.0;
      if ((fl[t] & 1u) && (s2[t] - E2 > tq || s2[t] + E2 < tq)) {
        if (s2[t] - E2 > tq && lane == 0) gadd(q.cnt + pi[t], 1);
        fl[t] &= ~1u;
      }
      if ((fl[t] & 2u) && (s2[t] - E2 > tg || s2[t] + E2 < tg)) {
        if (s2[t] - E2 > tg && lane == 0) gadd(g.cnt + pj[t], 1);
        fl[t] &= ~2u;
      }
      if (!fl[t]) continue;
      // level 3: fp64, the fix-up's arithmetic
      const double sc = wave_cos64((const TQ*)q.raw + pi[t] * q.ld, (const TG*)g.raw + pj[t] * g.ld,
                                   gld(q.inv + pi[t]), gld(g.inv + pj[t]), c.d, lane);
      if (lane == 0) {
        if ((fl[t] & 1u) && sc > tq) gadd(q.cnt + pi[t], 1);
        if ((fl[t] & 2u) && sc > tg) gadd(g.cnt + pj[t], 1);
      }
    }
  }
}

// the evaluation's fix-up: the listed undecided pairs -- with the level-2 planes eval_fix2_walk, else fp64
// (fixup_walk's flat walk)
template <typename TQ, typename TG>
__device__ __forceinline__ void eval_fix_body(const EvalSide& q, const EvalSide& g, const EvalCommon& c) {
  EVAL_STAMP(c, 2, 0);
  if (c.dbg & 8) {
  } else if (q.lo16 && g.lo16 && c.nb <= FIXUP_MAX_BUCKETS_PER_XCD) {
    eval_fix2_walk<TQ, TG>(q, g, c, blockIdx.x, gridDim.x);
  } else {
    fixup_walk<TQ, TG, true>((const TQ*)q.raw, q.ld, q.inv, (const TG*)g.raw, g.ld, g.inv, c.d, q.off ? q.sgt : nullptr,
                             g.off ? g.sgt : nullptr, q.cnt, g.cnt, c.cand, c.nb, c.cap_b,
                             c.nb <= FIXUP_MAX_BUCKETS_PER_XCD);
  }
  EVAL_STAMP(c, 2, 1);
}
template <typename TQ, typename TG>
__global__ __launch_bounds__(FIX_NT) void eval_fix_kernel(EvalSide q, EvalSide g, EvalCommon c) {
  eval_fix_body<TQ, TG>(q, g, c);
}
template <typename TQ, typename TG>
__global__ __launch_bounds__(FIX_NT) void eval_fix_batch_kernel(const EvalItem* __restrict__ tab) {
  const EvalItem& it = tab[blockIdx.y];
  eval_fix_body<TQ, TG>(it.q, it.g, it.c);
}

// the pair total / overflow size (cand_finalize_kernel's), one block
__device__ __forceinline__ void finish_buckets(const EvalCommon& c) {
  __shared__ unsigned long long redt[2 * FIN_NW], redm[2 * FIN_NW];
  unsigned long long tot[1] = {0}, mx[1] = {0};
  for (int64_t b = threadIdx.x; b < c.nb; b += FIN_NT) {
    const unsigned long long v = gld(c.bucket + b);
    tot[0] += v;
    mx[0] = v > mx[0] ? v : mx[0];
  }
  block_reduce_k<false>(tot, redt);
  block_reduce_k<true>(mx, redm);
  if (threadIdx.x == 0) {
    gst(c.stats + 8, (int64_t)tot[0]);
    gst(c.stats + 12, c.l3_count ? (int64_t)gld(c.l3_count) : 0);  // level-3 pairs (past l3_cap: re-scored inline)
    gst(c.stats + 9, (!c.fix_inline && (int64_t)mx[0] > c.cap_b) ? ((int64_t)mx[0] + 1) * c.nb + c.nb + 1 : 0);
  }
}

// err_max of both sides (all three planes, real rows, NaN skipped: err_max_kernel's result) as
// cmve_pack_rows leaves it, folded from the prep's shards, which are zeroed for the next evaluation
// (the rank GEMM has read them); one block
__device__ __forceinline__ void finish_err_max(const EvalSide& q, const EvalSide& g, const EvalCommon& c) {
  // one wave per (side, plane): each lane reads one of its 64 shards (one round of loads, not 64 serial
  // ones), a wave max, and zeroes the word it read
  static_assert(EMAX_SHARDS == 64, "one shard per lane");
  const int lane = threadIdx.x & 63;
  for (int sp = threadIdx.x >> 6; sp < 6; sp += FIN_NW) {
    unsigned* w = &c.emax[sp * EMAX_SHARDS + lane];
    unsigned m = gld(w);
    gst(w, 0u);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, 64));
    if (lane == 0) gst((sp < 3 ? q.err_max : g.err_max) + sp % 3, __uint_as_float(m));
  }
}

// The ranks of both directions (cmve_gt_ranks' rules) for this block's 256 rows of each side and, per
// direction, #rank<=1, <=5, <=10 and the rank sum, added into the stats head (zeroed by the prep)
template <typename TQ, typename TG, bool LIGHT = false>
__device__ __forceinline__ void eval_finish_body(const EvalSide& q, const EvalSide& g, const EvalCommon& c, int64_t vb,
                                                 int64_t nvb) {
  // vb / nvb: this block and the finish's block count (eval_prep_pair_f16_body's convention)
  EVAL_STAMP(c, 1, 0);
  if (c.dbg & 32) return;
  __shared__ unsigned long long red[9 * FIN_NW];
  const int64_t nrank = nvb - 2;  // the last two blocks: pair total / overflow, err_max
  if (vb >= nrank) {
    if (vb == nrank) finish_buckets(c);
    else finish_err_max(q, g, c);
    EVAL_STAMP(c, 1, 1);
    return;
  }
  // per wave: #rank <= 1 / 5 / 10 from ballots (no reduction), the rank sums in one butterfly of both
  // directions; then one LDS round over the block's waves and 8 lanes adding into the stats head
  const int64_t i = (int64_t)vb * FIN_NT + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // level 3, deferred by the rank GEMM (EvalCommon::l3): the listed pairs whose row (t2v) or column (v2t) is one
  // of this block's, re-scored in fp64 by wave_cos64 (the fix-up's arithmetic: the same bits as an inline
  // re-score) and added to this block's counts through LDS.  A pair listed for both directions is scored by
  // the block of its row and by the block of its column.
  __shared__ int add_q[FIN_NT], add_g[FIN_NT];
  // every load that does not depend on the level-3 pass first, with the list's count and each wave's first entry
  // (read speculatively: the list holds l3_cap entries), so the pass adds one round trip instead of three
  const bool hq = q.off && i < q.n, hg = g.off && i < g.n;
  int cq = 0, cg = 0, g1 = 0;
  double tq = 0.0, tg = 0.0;
  if (hq) {
    cq = gld(q.cnt + i);
    tq = gld(q.sgt + i);
    if (q.gt1) g1 = gld(q.gt1 + i);
  }
  if (hg) {
    cg = gld(g.cnt + i);
    tg = gld(g.sgt + i);
  }
  const bool l3 = c.l3_count != nullptr && FIN_NW <= c.l3_cap;
  const unsigned n3 = l3 ? min(gld(c.l3_count), (unsigned)c.l3_cap) : 0u;
  const uint64_t u_first = l3 ? gld(c.l3 + wave) : 0ull;
  if (n3) {
    add_q[threadIdx.x] = 0;
    add_g[threadIdx.x] = 0;
    __syncthreads();
    const int64_t r0 = (int64_t)vb * FIN_NT;
    for (unsigned e = (unsigned)wave; e < n3; e += FIN_NW) {
      const uint64_t u = e == (unsigned)wave ? u_first : gld(c.l3 + e);
      const int64_t pi = (int64_t)(u & 0x7fffffffull), pj = (int64_t)((u >> 31) & 0x7fffffffull);
      const unsigned fl = (unsigned)(u >> 62);
      const bool mq = (fl & 1u) && pi >= r0 && pi < r0 + FIN_NT;
      const bool mg = (fl & 2u) && pj >= r0 && pj < r0 + FIN_NT;
      if (!(mq || mg)) continue;  // (wave-uniform)
      const double sc = wave_cos64<TQ, TG, LIGHT>((const TQ*)q.raw + pi * q.ld, (const TG*)g.raw + pj * g.ld, gld(q.inv + pi),
                                   gld(g.inv + pj), c.d, lane);
      if (lane == 0) {
        if (mq && sc > gld(q.sgt + pi)) atomicAdd(&add_q[pi - r0], 1);
        if (mg && sc > gld(g.sgt + pj)) atomicAdd(&add_g[pj - r0], 1);
      }
    }
    __syncthreads();
  }
  int64_t rq = 0, rg = 0;
  bool unpaired = false;  // a CMVE_EVAL_PAIRED row whose lists were not a one-to-one pairing (the paired prep)
  if (hq) {
    rq = gt_rank_of(cq + (n3 ? add_q[threadIdx.x] : 0), tq, g.n);
    gst(q.ranks + i, rq);
    unpaired = q.gt1 && g1 == -2;
  }
  const unsigned long long unp = __builtin_amdgcn_ballot_w64(unpaired);
  if (unp && lane == 0) gadd((unsigned long long*)&c.stats[11], (unsigned long long)__builtin_popcountll(unp));
  if (hg) {
    rg = gt_rank_of(cg + (n3 ? add_g[threadIdx.x] : 0), tg, q.n);
    gst(g.ranks + i, rg);
  }
  unsigned long long sq = (unsigned long long)rq, sg = (unsigned long long)rg;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    sq += __shfl_xor(sq, o, 64);
    sg += __shfl_xor(sg, o, 64);
  }
  const unsigned long long w[8] = {
      (unsigned long long)__builtin_popcountll(__builtin_amdgcn_ballot_w64(rq != 0 && rq <= 1)),
      (unsigned long long)__builtin_popcountll(__builtin_amdgcn_ballot_w64(rq != 0 && rq <= 5)),
      (unsigned long long)__builtin_popcountll(__builtin_amdgcn_ballot_w64(rq != 0 && rq <= 10)), sq,
      (unsigned long long)__builtin_popcountll(__builtin_amdgcn_ballot_w64(rg != 0 && rg <= 1)),
      (unsigned long long)__builtin_popcountll(__builtin_amdgcn_ballot_w64(rg != 0 && rg <= 5)),
      (unsigned long long)__builtin_popcountll(__builtin_amdgcn_ballot_w64(rg != 0 && rg <= 10)), sg};
  if (lane < 8) {
    unsigned long long v = w[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) v = lane == k ? w[k] : v;
    red[lane * FIN_NW + wave] = v;
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    const int k = threadIdx.x;
    unsigned long long a = red[k * FIN_NW];
#pragma unroll
    for (int ww = 1; ww < FIN_NW; ++ww) a += red[k * FIN_NW + ww];
    if ((k < 4 ? q.off : g.off) && a) gadd((unsigned long long*)&c.stats[k], a);
  }
  EVAL_STAMP(c, 1, 1);
}

// entry kernels: one evaluation (arguments by value), or a batch of same-shaped evaluations whose argument
// blocks sit in a device table (cmve_eval_batch_*: blockIdx.y = the evaluation; the bodies index blocks by x)
template <typename TQ, typename TG>
__global__ __launch_bounds__(PREP_NT) void eval_prep_kernel(EvalSide q, EvalSide g, EvalCommon c) {
  eval_prep_body<TQ, TG>(q, g, c);
}
template <typename TQ, typename TG>
__global__ __launch_bounds__(PREP_NT) void eval_prep_pair_kernel(EvalSide q, EvalSide g, EvalCommon c) {
  eval_prep_pair_body<TQ, TG>(q, g, c);
}
template <typename TQ, typename TG>
__global__ __launch_bounds__(FIN_NT) void eval_finish_kernel(EvalSide q, EvalSide g, EvalCommon c) {
  eval_finish_body<TQ, TG>(q, g, c, blockIdx.x, gridDim.x);
}
template <typename TQ, typename TG>
__global__ __launch_bounds__(PREP_NT) void eval_prep_batch_kernel(const EvalItem* __restrict__ tab) {
  const EvalItem& it = tab[blockIdx.y];
  eval_prep_body<TQ, TG>(it.q, it.g, it.c);
}
template <typename TQ, typename TG>
__global__ __launch_bounds__(PREP_NT) void eval_prep_pair_batch_kernel(const EvalItem* __restrict__ tab) {
  const EvalItem& it = tab[blockIdx.y];
  eval_prep_pair_body<TQ, TG>(it.q, it.g, it.c);
}
#ifndef CMVE_PREP_WPE
#define CMVE_PREP_WPE 4  // the specialized paired prep: waves per SIMD its register budget allows (<= 128 VGPRs)
#endif
template <typename TQ, typename TG, int NM>
__global__ __launch_bounds__(PREP_NT, CMVE_PREP_WPE) void eval_prep_pair_f16_kernel(EvalSide q, EvalSide g, EvalCommon c) {
  eval_prep_pair_f16_body<TQ, TG, NM>(q, g, c, blockIdx.x, gridDim.x);
}
template <typename TQ, typename TG, int NM>
__global__ __launch_bounds__(PREP_NT, CMVE_PREP_WPE) void eval_prep_pair_f16_batch_kernel(const EvalItem* __restrict__ tab) {
  const EvalItem& it = tab[blockIdx.y];
  eval_prep_pair_f16_body<TQ, TG, NM>(it.q, it.g, it.c, blockIdx.x, gridDim.x);
}
template <typename TQ, typename TG>
__global__ __launch_bounds__(FIN_NT) void eval_finish_batch_kernel(const EvalItem* __restrict__ tab) {
  const EvalItem& it = tab[blockIdx.y];
  eval_finish_body<TQ, TG>(it.q, it.g, it.c, blockIdx.x, gridDim.x);
}
// The chained batch launch (cmve_eval_batch_run_chained): the specialised prep of a batch and the finish of the
// batch run before it on the same stream in ONE launch -- row y of the grid: blocks [0, nprep) the prep of
// evaluation y of ptab, blocks [nprep, nprep + nfin) the finish of evaluation y of ftab (no ftab: those blocks
// return).  The two roles touch different workspaces (the caller checks), and the finish's inputs were complete
// when the previous batch's rank GEMM ended, before this launch: one launch per batch fewer on the stream, and
// the finish's few blocks run in the prep's shadow instead of as a launch of their own between two batches.
template <typename TQ, typename TG, int NM>
#ifndef CMVE_PREPFIN_WPE
#define CMVE_PREPFIN_WPE 4  // (the finish role takes the light fp64 re-score: the full one alone took 114 registers,
#endif                      // and a launch above 104 fits one wave per SIMD beside the batch rank GEMM's two, not two)
__global__ __launch_bounds__(PREP_NT, CMVE_PREPFIN_WPE) void eval_prep_fin_batch_kernel(const EvalItem* __restrict__ ptab,
                                                                                    const EvalItem* __restrict__ ftab,
                                                                                    int nprep, int nfin,
                                                                                    const EvalItem* __restrict__ xtab,
                                                                                    int nfix) {
  static_assert(PREP_NT == FIN_NT && PREP_NT == FIX_NT, "one block size for every role");
#ifdef CMVE_STUDY_PREP_PRIO  // study: the chained prep's waves at a raised priority beside another stream's rank GEMM
  __builtin_amdgcn_s_setprio(CMVE_STUDY_PREP_PRIO);
#endif
  const int bx = (int)blockIdx.x;
  if (bx < nprep) {
    const EvalItem& it = ptab[blockIdx.y];
    eval_prep_pair_f16_body<TQ, TG, NM>(it.q, it.g, it.c, blockIdx.x, nprep);
  } else if (bx < nprep + nfin) {
    const EvalItem& it = ftab[blockIdx.y];
    eval_finish_body<TQ, TG, true>(it.q, it.g, it.c, bx - nprep, nfin);
  } else {
#if CMVE_EVAL_FIX_CHAINED  // study: the previous batch's level-2 / fp64 fix-up as a third role of the launch
    const EvalItem& it = xtab[blockIdx.y];
    eval_fix2_walk<TQ, TG, EVAL_FIXC_MAXB>(it.q, it.g, it.c, bx - nprep - nfin, nfix);
#else
    (void)xtab;
    (void)nfix;
#endif
  }
}

// the specialized paired prep applies: F16 with the lo16 plane, 16-B row pieces, d = d_pad = 256 NM (NM <= 4)
static int prep_f16_nm(const EvalSide& q, const EvalSide& g, const EvalCommon& c) {
  const bool ok = c.mode == CMVE_SIM_F16 && q.h16 && g.h16 && q.lo16 && g.lo16 && q.vec && g.vec && c.d == c.d_pad &&
                  c.d_pad % 256 == 0 && c.d_pad <= 1024;
  return ok ? (int)(c.d_pad / 256) : 0;
}
#define CMVE_PREP_F16(KER, NMV, ...)                                                                            \
  switch (NMV) {                                                                                                \
    case 1: cmve::launch(KER<TQ, TG, 1>, __VA_ARGS__); break;                                                  \
    case 2: cmve::launch(KER<TQ, TG, 2>, __VA_ARGS__); break;                                                  \
    case 3: cmve::launch(KER<TQ, TG, 3>, __VA_ARGS__); break;                                                  \
    default: cmve::launch(KER<TQ, TG, 4>, __VA_ARGS__); break;                                                 \
  }

template <typename TQ, typename TG>
static int launch_eval_batch_typed(const EvalSide& q, const EvalSide& g, const EvalCommon& c0, const EvalItem* tab,
                                   int count, int phase, hipStream_t s) {
  if (phase == 0) {
    const unsigned blocks = (unsigned)((q.n_pad + g.n_pad + PREP_NW - 1) / PREP_NW);
    cmve::launch(eval_prep_batch_kernel<TQ, TG>, dim3(blocks, (unsigned)count), dim3(PREP_NT), 0u, s, tab);
    return check_launch("eval_prep_batch_kernel");
  }
  if (phase == 1) {
    // the batch's fix-up: CMVE_FIXB_BLOCKS blocks of 4 waves per evaluation (~1,600 listed pairs at 1k-A)
    cmve::launch(eval_fix_batch_kernel<TQ, TG>, dim3((unsigned)CMVE_FIXB_BLOCKS, (unsigned)count), dim3(FIX_NT), 0u,
                 s, tab);
    return check_launch("eval_fix_batch_kernel");
  }
  if (phase == 3) {
    const unsigned blocks = (unsigned)((q.n_pad + PREP_NW - 1) / PREP_NW);
    if (const int nm = prep_f16_nm(q, g, c0)) {
      CMVE_PREP_F16(eval_prep_pair_f16_batch_kernel, nm, dim3(blocks, (unsigned)count), dim3(PREP_NT), 0u, s, tab);
      return check_launch("eval_prep_pair_f16_batch_kernel");
    }
    cmve::launch(eval_prep_pair_batch_kernel<TQ, TG>, dim3(blocks, (unsigned)count), dim3(PREP_NT), 0u, s, tab);
    return check_launch("eval_prep_pair_batch_kernel");
  }
  const int64_t nmax = q.n > g.n ? q.n : g.n;
  cmve::launch(eval_finish_batch_kernel<TQ, TG>, dim3((unsigned)((nmax + FIN_NT - 1) / FIN_NT) + 2, (unsigned)count),
               dim3(FIN_NT), 0u, s, tab);
  return check_launch("eval_finish_batch_kernel");
}

template <typename TQ, typename TG>
static int launch_eval_batch_chained_typed(const EvalSide& q, const EvalSide& g, const EvalCommon& c0,
                                           const EvalItem* ptab, const EvalItem* ftab, int count, hipStream_t s,
                                           const EvalItem* xtab) {
  const int nm = prep_f16_nm(q, g, c0);
  CMVE_REQUIRE(nm, "launch_eval_batch_chained: the batch does not take the specialised paired prep");
  CMVE_REQUIRE(!xtab || (CMVE_EVAL_FIX_CHAINED && c0.nb <= EVAL_FIXC_MAXB),
               "launch_eval_batch_chained: no fix-up role in this build / too many buckets");
  const int nprep = (int)((q.n_pad + PREP_NW - 1) / PREP_NW);
  const int64_t nmax = q.n > g.n ? q.n : g.n;
  const int nfin = ftab ? (int)((nmax + FIN_NT - 1) / FIN_NT) + 2 : 0;
  const int nfix = xtab ? CMVE_FIXB_BLOCKS : 0;
  CMVE_PREP_F16(eval_prep_fin_batch_kernel, nm, dim3((unsigned)(nprep + nfin + nfix), (unsigned)count),
                dim3(PREP_NT), 0u, s, ptab, ftab, nprep, nfin, xtab, nfix);
  return check_launch("eval_prep_fin_batch_kernel");
}

// the specialised paired prep of `ptab` and the finish of `ftab` (nullptr: none) in one launch; both batches have
// the shapes of q / g / c0 and `count` evaluations
int launch_eval_batch_chained(const EvalSide& q, const EvalSide& g, const EvalCommon& c0, const EvalItem* ptab,
                              const EvalItem* ftab, int count, int q_f64, int g_f64, hipStream_t s,
                              const EvalItem* xtab) {
  if (!q_f64 && !g_f64) return launch_eval_batch_chained_typed<float, float>(q, g, c0, ptab, ftab, count, s, xtab);
  if (!q_f64 && g_f64) return launch_eval_batch_chained_typed<float, double>(q, g, c0, ptab, ftab, count, s, xtab);
  if (q_f64 && !g_f64) return launch_eval_batch_chained_typed<double, float>(q, g, c0, ptab, ftab, count, s, xtab);
  return launch_eval_batch_chained_typed<double, double>(q, g, c0, ptab, ftab, count, s, xtab);
}

// whether a batch of these shapes takes launch_eval_batch_chained
bool eval_batch_chainable(const EvalSide& q, const EvalSide& g, const EvalCommon& c0) { return prep_f16_nm(q, g, c0) != 0; }

// a batch: the items share q / g shapes, dtypes and GT lists (tab[i] differ in buffers only); phases 0 / 2 / 3
// as launch_eval (no separate fix-up: the batch path is the G64 inline fix-up geometry)
int launch_eval_batch(const EvalSide& q, const EvalSide& g, const EvalCommon& c0, const EvalItem* tab, int count,
                      int q_f64, int g_f64, int phase, hipStream_t s) {
  if (!q_f64 && !g_f64) return launch_eval_batch_typed<float, float>(q, g, c0, tab, count, phase, s);
  if (!q_f64 && g_f64) return launch_eval_batch_typed<float, double>(q, g, c0, tab, count, phase, s);
  if (q_f64 && !g_f64) return launch_eval_batch_typed<double, float>(q, g, c0, tab, count, phase, s);
  return launch_eval_batch_typed<double, double>(q, g, c0, tab, count, phase, s);
}

template <typename TQ, typename TG>
static int launch_eval_typed(const EvalSide& q, const EvalSide& g, const EvalCommon& c, int phase, hipStream_t s) {
  if (phase == 0) {
    const unsigned blocks = (unsigned)((q.n_pad + g.n_pad + PREP_NW - 1) / PREP_NW);
    cmve::launch(eval_prep_kernel<TQ, TG>, dim3(blocks), dim3(PREP_NT), 0u, s, q, g, c);
    return check_launch("eval_prep_kernel");
  }
  if (phase == 3) {  // the paired prep (eval_prep_pair_kernel): one wave per (caption, video) pair
    const unsigned blocks = (unsigned)((q.n_pad + PREP_NW - 1) / PREP_NW);
    if (const int nm = prep_f16_nm(q, g, c)) {
      CMVE_PREP_F16(eval_prep_pair_f16_kernel, nm, dim3(blocks), dim3(PREP_NT), 0u, s, q, g, c);
      return check_launch("eval_prep_pair_f16_kernel");
    }
    cmve::launch(eval_prep_pair_kernel<TQ, TG>, dim3(blocks), dim3(PREP_NT), 0u, s, q, g, c);
    return check_launch("eval_prep_pair_kernel");
  }
  if (phase == 1) {
    // 1,024 blocks of 4 waves, every wave one or two of the few thousand undecided pairs of an evaluation
    // of this size, in one flat walk (the rank fix-up's grid is sized for millions of pairs)
    cmve::launch(eval_fix_kernel<TQ, TG>, dim3((unsigned)CMVE_FIX_BLOCKS), dim3(FIX_NT), 0u, s, q, g, c);
    return check_launch("eval_fix_kernel");
  }
  const int64_t nmax = q.n > g.n ? q.n : g.n;
  cmve::launch(eval_finish_kernel<TQ, TG>, dim3((unsigned)((nmax + FIN_NT - 1) / FIN_NT) + 2), dim3(FIN_NT), 0u, s,
               q, g, c);
  return check_launch("eval_finish_kernel");
}

// phase 0: prep, phase 1: fix-up, phase 2: err_max + ranks + R@K, phase 3: the paired prep
int launch_eval(const EvalSide& q, const EvalSide& g, const EvalCommon& c, int q_f64, int g_f64, int phase,
                hipStream_t s) {
  if (!q_f64 && !g_f64) return launch_eval_typed<float, float>(q, g, c, phase, s);
  if (!q_f64 && g_f64) return launch_eval_typed<float, double>(q, g, c, phase, s);
  if (q_f64 && !g_f64) return launch_eval_typed<double, float>(q, g, c, phase, s);
  return launch_eval_typed<double, double>(q, g, c, phase, s);
}

}  // namespace cmve
