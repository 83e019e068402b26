// K5: exact fp64 GT scores / rank thresholds and the fp64 fix-up of undecided pairs,
// plus rank counting from a given error matrix (eval_q2m on a materialised matrix).
//
// The reference scores in float64 (LINAS-engine/evaluation.py:102,105 store the
// embeddings in np.zeros -> float64; evaluation.py:18-21 normalises and dots in
// float64) and ranks with np.argsort (LINAS-engine/util/metrics.py:137-147).  The
// canonical exact score used here is
//     cos64(x, y) = dot64(raw_x, raw_y) * (inv_norm_x * inv_norm_y)
// which is symmetric in (x, y): the GT-score kernel and the fix-up kernel compute a
// given pair bit-identically whichever side is the query.
#include "cmve_internal.h"

namespace cmve {

template <typename TA, typename TB>
__device__ __forceinline__ double cos64(const TA* xa, const TB* xb, double inva, double invb, int64_t d, int lane) {
  return wave_dot64(xa, xb, d, lane) * (inva * invb);
}

template <typename TA, typename TB>
__global__ __launch_bounds__(256) void gt_thr_kernel(const TA* __restrict__ araw, int64_t lda,
                                                     const double* __restrict__ ainv, const float* __restrict__ aerr,
                                                     int64_t na, int64_t na_pad, const TB* __restrict__ braw,
                                                     int64_t ldb, const double* __restrict__ binv,
                                                     const float* __restrict__ berr_max, int64_t d, int64_t d_pad,
                                                     int mode, const int64_t* __restrict__ off,
                                                     const int32_t* __restrict__ idx, double* __restrict__ sgt,
                                                     float* __restrict__ thr_hi, float* __restrict__ thr_lo) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= na_pad) return;
  if (row >= na) {
    if (lane == 0) {
      sgt[row] = NAN;
      thr_hi[row] = INFINITY;
      thr_lo[row] = INFINITY;
    }
    return;
  }
  double best = -INFINITY;
  bool any = false;
  const TA* xa = araw + row * lda;
  for (int64_t k = off[row]; k < off[row + 1]; ++k) {
    const int64_t b = idx[k];
    const double s = cos64(xa, braw + b * ldb, ainv[row], binv[b], d, lane);
    if (s == s) {
      any = true;
      if (s > best) best = s;
    }
  }
  if (lane == 0) {
    if (!any) {
      // Never counted.  Empty GT list: sgt = NaN (rank n_m + 1, metrics.py:140).  A non-empty list
      // whose every GT scores NaN (zero-norm row, no eps in l2norm): sgt = +inf (rank n_m -- np.argsort
      // puts NaN after every finite score; see cmve_gt_ranks for the rule among several NaN).
      sgt[row] = off[row + 1] > off[row] ? (double)INFINITY : (double)NAN;
      thr_hi[row] = INFINITY;
      thr_lo[row] = INFINITY;
    } else {
      const double E = score_error_bound((double)aerr[row], (double)berr_max[mode_slot(mode)], d_pad,
                                         mode);
      sgt[row] = best;
      thr_hi[row] = f32_round_up(best + E);
      thr_lo[row] = f32_round_down(best - E);
    }
  }
}

// thresholds from given exact GT scores (sharded path: sgt computed by the GT's owner rank)
__global__ __launch_bounds__(256) void thr_from_sgt_kernel(const double* __restrict__ sgt, const float* __restrict__ aerr,
                                                           int64_t na, int64_t na_pad,
                                                           const float* __restrict__ berr_max, int64_t d_pad, int mode,
                                                           float* __restrict__ thr_hi, float* __restrict__ thr_lo) {
  const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (row >= na_pad) return;
  const double s = row < na ? sgt[row] : NAN;
  if (!(s < INFINITY)) {  // NaN (no GT) or +inf (every GT scores NaN): never counted
    thr_hi[row] = INFINITY;
    thr_lo[row] = INFINITY;
    return;
  }
  const double E = score_error_bound((double)aerr[row], (double)berr_max[mode_slot(mode)], d_pad, mode);
  thr_hi[row] = f32_round_up(s + E);
  thr_lo[row] = f32_round_down(s - E);
}

// *cand_count = total pairs, or -- if a bucket outgrew cap_b (or cand is NULL: the buffer cannot
// hold the counters) -- a size > cand_cap that fits the largest bucket, so the caller's
// grow-and-retry allocates enough.
__global__ __launch_bounds__(256) void cand_finalize_kernel(const uint64_t* __restrict__ bcnt, int64_t nb,
                                                            int64_t cap_b, int64_t cap, int64_t* __restrict__ out) {
  __shared__ unsigned long long s_tot[4], s_max[4];
  unsigned long long tot = 0, mx = 0;
  if (bcnt)
    for (int64_t b = threadIdx.x; b < nb; b += 256) {
      const unsigned long long c = bcnt[b];
      tot += c;
      mx = c > mx ? c : mx;
    }
  for (int o = 32; o >= 1; o >>= 1) {
    tot += __shfl_xor(tot, o, 64);
    const unsigned long long m2 = __shfl_xor(mx, o, 64);
    mx = m2 > mx ? m2 : mx;
  }
  if ((threadIdx.x & 63) == 0) {
    s_tot[threadIdx.x >> 6] = tot;
    s_max[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    tot = s_tot[0] + s_tot[1] + s_tot[2] + s_tot[3];
    mx = max(max(s_max[0], s_max[1]), max(s_max[2], s_max[3]));
    if (!bcnt || (int64_t)mx > cap_b) {
      const int64_t need = ((int64_t)mx + 1) * nb + nb + 1;
      *out = need > cap ? need : cap + 1;
    } else {
      *out = (int64_t)tot;
    }
  }
}

int launch_cand_finalize(hipStream_t stream, const cmve_rows_t* g, uint64_t* cand, int64_t cand_cap,
                         int64_t* cand_count) {
  const CandLayout l = cand_layout(g->n_pad, cand_cap);
  hipLaunchKernelGGL(cand_finalize_kernel, dim3(1), dim3(256), 0, stream, (const uint64_t*)cand, l.nb, l.cap_b,
                     cand_cap, cand_count);
  return check_launch("cand_finalize");
}

// XCD-ordered re-score of the bucketed undecided pairs (fixup_walk, cmve_internal.h)
template <typename TQ, typename TG, bool PF>
__global__ __launch_bounds__(256) void fixup_kernel(const TQ* __restrict__ qraw, int64_t ldq,
                                                    const double* __restrict__ qinv, const TG* __restrict__ graw,
                                                    int64_t ldg, const double* __restrict__ ginv, int64_t d,
                                                    const double* __restrict__ row_sgt,
                                                    const double* __restrict__ col_sgt, int* __restrict__ row_cnt,
                                                    int* __restrict__ col_cnt, const uint64_t* __restrict__ cand,
                                                    int64_t nb, int64_t cap_b) {
  fixup_walk<TQ, TG, PF, true, true>(qraw, ldq, qinv, graw, ldg, ginv, d, row_sgt, col_sgt, row_cnt, col_cnt, cand, nb,
                                     cap_b, false);
}

// the walk over nb buckets of cap_b entries at cand (counts at cand[0, nb)).  Every wave has one pair in flight.
// Rows under 4 KiB (C4's 640-d fp32): as many blocks as the registers let the CUs hold (24 waves per CU), since the
// walk is bound by the round trips in flight there (C4 ranking 10.1 -> 8.5 ms; it used to be held to 16 waves per
// CU by a 32 KiB static LDS prefix).  Wider rows (the 1024-d gallery shards: a query row per pair from the
// Infinity Cache at ~6 TB/s) keep 128 blocks per XCD: more waves in flight only contend (1M-gallery fix-up 11.6 ->
// 13.4 ms).  Study builds: CMVE_FIX_BPX (blocks per XCD), CMVE_FIX_PF=1 (GT scores loaded ahead of the dot).
#ifndef CMVE_FIX_BPX
#define CMVE_FIX_BPX 0
#endif
#ifndef CMVE_FIX_PF
#define CMVE_FIX_PF 0
#endif
template <typename TQ, typename TG, bool PF>
static void launch_fix(hipStream_t stream, const cmve_rows_t* q, const cmve_rows_t* g, const double* row_sgt,
                       const double* col_sgt, int32_t* row_cnt, int32_t* col_cnt, const uint64_t* cand, int64_t nb,
                       int64_t cap_b) {
  static const int per_cu = [] {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)fixup_kernel<TQ, TG, PF>, 256, 512) != hipSuccess)
      n = 4;
    return std::max(1, n);
  }();
  const int64_t row_bytes = q->d * std::max<int64_t>(sizeof(TQ), sizeof(TG));
  const int bpx = CMVE_FIX_BPX > 0 ? std::min(1024, CMVE_FIX_BPX)
                  : row_bytes < 4096 ? per_cu * std::max(1, device_cus() / 8) : 128;
  const unsigned lds = (unsigned)(((nb + 7) / 8 + 1) * sizeof(int64_t));  // the walk's bucket prefix
  hipLaunchKernelGGL((fixup_kernel<TQ, TG, PF>), dim3(8u * (unsigned)bpx), dim3(256), lds, stream, (const TQ*)q->raw,
                     q->raw_ld, q->inv_norm, (const TG*)g->raw, g->raw_ld, g->inv_norm, q->d, row_sgt, col_sgt, row_cnt,
                     col_cnt, cand, nb, cap_b);
}

static int launch_fixup_walk(hipStream_t stream, const cmve_rows_t* q, const cmve_rows_t* g, const double* row_sgt,
                             const double* col_sgt, int32_t* row_cnt, int32_t* col_cnt, const uint64_t* cand,
                             int64_t nb, int64_t cap_b) {
  constexpr bool PF = CMVE_FIX_PF != 0;
#define FIX(TQ, TG) launch_fix<TQ, TG, PF>(stream, q, g, row_sgt, col_sgt, row_cnt, col_cnt, cand, nb, cap_b)
  if (q->raw_dtype == CMVE_F32 && g->raw_dtype == CMVE_F32) FIX(float, float);
  else if (q->raw_dtype == CMVE_F32 && g->raw_dtype == CMVE_F64) FIX(float, double);
  else if (q->raw_dtype == CMVE_F64 && g->raw_dtype == CMVE_F32) FIX(double, float);
  else FIX(double, double);
#undef FIX
  return check_launch("fixup_kernel");
}

int launch_fixup(hipStream_t stream, const cmve_rows_t* q, const cmve_rows_t* g, int32_t dirs, const double* row_sgt,
                 const double* col_sgt, int32_t* row_cnt, int32_t* col_cnt, const uint64_t* cand, int64_t cand_cap,
                 const int64_t* cand_count) {
  (void)cand_count;  // the bucket counters at the head of `cand` carry the sizes
  const CandLayout l = cand_layout(g->n_pad, cand_cap);
  if (l.cap_b == 0) return CMVE_OK;  // reported as overflow by the MFMA pass: the caller retries
  CMVE_REQUIRE((l.nb + 7) / 8 <= FIXUP_MAX_BUCKETS_PER_XCD, "cmve_rank_fixup: gallery set too large (%lld buckets)",
               (long long)l.nb);
  // a disabled direction has flags that never set its bit; pass its (possibly NULL) arrays through
  (void)dirs;
  return launch_fixup_walk(stream, q, g, row_sgt, col_sgt, row_cnt, col_cnt, cand, l.nb, l.cap_b);
}

// ---- rank from a materialised error matrix (lower = better) ----
template <typename T>
__global__ __launch_bounds__(256) void rank_rows_kernel(const T* __restrict__ e, int64_t n_cols, int64_t ld,
                                                        const int64_t* __restrict__ off,
                                                        const int32_t* __restrict__ idx, int32_t* __restrict__ cnt) {
  __shared__ int part[4];
  const int64_t row = blockIdx.x;
  const T* er = e + row * ld;
  double thr = INFINITY;
  bool any = false;
  for (int64_t k = off[row]; k < off[row + 1]; ++k) {
    const double v = (double)er[idx[k]];
    if (v == v) {
      any = true;
      if (v < thr) thr = v;
    }
  }
  int c = 0;
  if (any)
    for (int64_t j = threadIdx.x; j < n_cols; j += 256) c += ((double)er[j] < thr);
  c = wave_sum_i(c);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  // every GT NaN: rank n_m (NaN sorts last; the GT taken as the last of the row's NaN entries)
  if (threadIdx.x == 0)
    cnt[row] = (!any && off[row + 1] > off[row]) ? (int32_t)(n_cols - 1) : part[0] + part[1] + part[2] + part[3];
}

// columns of e ranked (the errors.T view): thread per column, rows split over blockIdx.y
template <typename T>
__global__ __launch_bounds__(256) void rank_cols_kernel(const T* __restrict__ e, int64_t n_rows, int64_t n_cols,
                                                        int64_t ld, int64_t rows_per_split,
                                                        const int64_t* __restrict__ off,
                                                        const int32_t* __restrict__ idx, int32_t* __restrict__ cnt) {
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (col >= n_cols) return;
  double thr = INFINITY;
  bool any = false;
  for (int64_t k = off[col]; k < off[col + 1]; ++k) {
    const double v = (double)e[(int64_t)idx[k] * ld + col];
    if (v == v) {
      any = true;
      if (v < thr) thr = v;
    }
  }
  if (!any) {  // every GT NaN: rank n_m (counts are zeroed by the caller; one split adds n_rows - 1)
    if (blockIdx.y == 0 && off[col + 1] > off[col]) atomicAdd(&cnt[col], (int)(n_rows - 1));
    return;
  }
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_split;
  const int64_t r1 = r0 + rows_per_split < n_rows ? r0 + rows_per_split : n_rows;
  int c = 0;
  for (int64_t i = r0; i < r1; ++i) c += ((double)e[i * ld + col] < thr);
  if (c) atomicAdd(&cnt[col], c);
}

// Positions of EVERY GT item (for mAP, LINAS-engine/util/metrics.py:61-102):
//   pos[k] = #{ j : e_ij < e_{i, idx[k]} }  for k in [off[i], off[i+1])
// Rows: one block per row, GT values sorted in LDS, each element binary-searches
// the first GT value above it and bumps a histogram; prefix sums give the counts.
constexpr int MAXG = 64;

template <typename T>
__global__ __launch_bounds__(256) void gtpos_rows_kernel(const T* __restrict__ e, int64_t n_cols, int64_t ld,
                                                         const int64_t* __restrict__ off,
                                                         const int32_t* __restrict__ idx, int32_t* __restrict__ pos) {
  __shared__ double tv[MAXG];
  __shared__ int tk[MAXG];
  __shared__ int hist[MAXG + 1];
  const int64_t row = blockIdx.x;
  const T* er = e + row * ld;
  const int64_t k0 = off[row];
  const int m = (int)(off[row + 1] - k0);
  if (m == 0) return;
  // NaN GT items take the last positions of the row, n_cols - n_nan .. n_cols - 1 (np.argsort puts NaN
  // after every finite score; the order among several NaN is implementation-defined there, and AP
  // depends only on the set of positions)
  __shared__ int s_nan_total, s_nan_run;
  if (threadIdx.x == 0) {
    int nn = 0;
    for (int a = 0; a < m; ++a) {
      const double v = (double)er[idx[k0 + a]];
      nn += (v != v);
    }
    s_nan_total = nn;
    s_nan_run = 0;
  }
  for (int base = 0; base < m; base += MAXG) {  // GT lists longer than MAXG: chunks
    const int mc = min(MAXG, m - base);
    if (threadIdx.x == 0) {
      for (int a = 0; a < mc; ++a) {  // insertion sort ascending (NaN last)
        const double v = (double)er[idx[k0 + base + a]];
        int b = a;
        while (b > 0 && (tv[b - 1] > v || (tv[b - 1] != tv[b - 1] && v == v))) {
          tv[b] = tv[b - 1];
          tk[b] = tk[b - 1];
          --b;
        }
        tv[b] = v;
        tk[b] = a;
      }
    }
    for (int a = threadIdx.x; a <= MAXG; a += 256) hist[a] = 0;
    __syncthreads();
    for (int64_t j = threadIdx.x; j < n_cols; j += 256) {
      const double v = (double)er[j];
      if (v != v) continue;  // NaN is never "better"
      int lo = 0, hi = mc;   // first p with tv[p] > v (NaN thresholds compare false -> never beaten... treated as +inf)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const double t = tv[mid];
        if (t > v || t != t) hi = mid; else lo = mid + 1;
      }
      if (lo < mc) atomicAdd(&hist[lo], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int run = 0;
      for (int p = 0; p < mc; ++p) {
        run += hist[p];
        pos[k0 + base + tk[p]] = (tv[p] != tv[p]) ? (int)n_cols - s_nan_total + s_nan_run++ : run;
      }
    }
    __syncthreads();
  }
}

// columns (errors.T view): one block per 64 columns, 4 row-slices per block reduce in LDS
template <typename T>
__global__ __launch_bounds__(256) void gtpos_cols_kernel(const T* __restrict__ e, int64_t n_rows, int64_t n_cols,
                                                         int64_t ld, const int64_t* __restrict__ off,
                                                         const int32_t* __restrict__ idx, int32_t* __restrict__ pos) {
  const int lane = threadIdx.x & 63, slice = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + lane;
  const bool valid = col < n_cols;
  const int64_t k0 = valid ? off[col] : 0;
  const int m = valid ? (int)(off[col + 1] - k0) : 0;
  const int64_t rs0 = (n_rows * slice) / 4, rs1 = (n_rows * (slice + 1)) / 4;
  __shared__ int cnt[4][64];
  // every wave of the block holds the same 64 columns, so the trip count is block-uniform
  int m_max = m;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m_max = max(m_max, __shfl_xor(m_max, o, 64));
  // NaN GT items: the last positions, n_rows - n_nan .. n_rows - 1 (as gtpos_rows_kernel)
  int nan_total = 0, nan_run = 0;
  for (int a = 0; a < m; ++a) {
    const double t = (double)e[(int64_t)idx[k0 + a] * ld + col];
    nan_total += (t != t);
  }
  for (int a = 0; a < m_max; ++a) {
    int c = 0;
    if (a < m) {
      const double t = (double)e[(int64_t)idx[k0 + a] * ld + col];
      if (t == t)
        for (int64_t i = rs0; i < rs1; ++i) c += ((double)e[i * ld + col] < t);
      else
        c = -1;
    }
    cnt[slice][lane] = c;
    __syncthreads();
    if (slice == 0 && a < m) {
      const int c0 = cnt[0][lane];
      pos[k0 + a] = c0 < 0 ? (int)n_rows - nan_total + nan_run : c0 + cnt[1][lane] + cnt[2][lane] + cnt[3][lane];
    }
    if (a < m && cnt[0][lane] < 0) ++nan_run;
    __syncthreads();
  }
}

// 1-based GT ranks from better-than-GT counts (LINAS-engine/util/metrics.py:137-147 on tie-free rows):
//   sgt NaN  (empty GT list)        -> n_m + 1   (metrics.py:140 initialises rank = n_m + 1)
//   sgt +inf (every GT scores NaN)  -> n_m       (np.argsort puts NaN after every finite score; with
//                                                 several NaN in a row numpy's order among them is
//                                                 implementation-defined: the GT is taken as the last)
//   else                            -> cnt + 1
// recall (optional, one block): #(rank<=1), #(rank<=5), #(rank<=10), sum of ranks (metrics.py:149-157).
__global__ __launch_bounds__(1024) void gt_ranks_kernel(const int32_t* __restrict__ cnt,
                                                        const double* __restrict__ sgt, int64_t n, int64_t n_m,
                                                        int64_t* __restrict__ ranks,
                                                        unsigned long long* __restrict__ recall) {
  unsigned long long r1 = 0, r5 = 0, r10 = 0, sum = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = gt_rank_of(cnt[i], sgt[i], n_m);
    if (ranks) ranks[i] = r;
    r1 += (r <= 1);
    r5 += (r <= 5);
    r10 += (r <= 10);
    sum += (unsigned long long)r;
  }
  if (!recall) return;
  __shared__ unsigned long long part[16][4];
  for (int o = 32; o >= 1; o >>= 1) {
    r1 += __shfl_xor(r1, o, 64);
    r5 += __shfl_xor(r5, o, 64);
    r10 += __shfl_xor(r10, o, 64);
    sum += __shfl_xor(sum, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    part[w][0] = r1;
    part[w][1] = r5;
    part[w][2] = r10;
    part[w][3] = sum;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    unsigned long long t = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += part[k][threadIdx.x];
    recall[threadIdx.x] = t;
  }
}

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_gt_ranks(cmve_handle_t h, const int32_t* cnt, const double* sgt, int64_t n, int64_t n_m,
                             int64_t* ranks, int64_t* recall) {
  CMVE_REQUIRE(h && cnt && sgt, "cmve_gt_ranks: NULL argument");
  CMVE_REQUIRE(ranks || recall, "cmve_gt_ranks: no output");
  CMVE_REQUIRE(n >= 0 && n_m >= 0, "cmve_gt_ranks: bad size");
  if (n == 0) {
    if (recall) CMVE_HIP(hipMemsetAsync(recall, 0, 4 * sizeof(int64_t), h->stream));
    return CMVE_OK;
  }
  // the recall sums need one block; without them a grid over the rows
  const unsigned blocks = recall ? 1u : (unsigned)std::min<int64_t>((n + 1023) / 1024, 4096);
  hipLaunchKernelGGL(gt_ranks_kernel, dim3(blocks), dim3(1024), 0, h->stream, cnt, sgt, n, n_m, ranks,
                     (unsigned long long*)recall);
  return check_launch("gt_ranks_kernel");
}

extern "C" int cmve_gt_thresholds(cmve_handle_t h, const cmve_rows_t* a, const cmve_rows_t* b, int32_t mode,
                                  const int64_t* off, const int32_t* idx, double* sgt, float* thr_hi,
                                  float* thr_lo) {
  CMVE_REQUIRE(h && a && b, "cmve_gt_thresholds: NULL argument");
  CMVE_REQUIRE(a->d == b->d && a->d_pad == b->d_pad, "cmve_gt_thresholds: dimension mismatch");
  CMVE_REQUIRE(!((a->flags | b->flags) & CMVE_PACK_RAW), "cmve_gt_thresholds: sets packed CMVE_PACK_RAW have no score bound");
  CMVE_REQUIRE(mode == CMVE_SIM_BF16 || mode == CMVE_SIM_BF16X3 || mode == CMVE_SIM_F16,
               "cmve_gt_thresholds: unknown mode");
  CMVE_REQUIRE(off && sgt && thr_hi && thr_lo, "cmve_gt_thresholds: NULL output");
  CMVE_REQUIRE(a->n == 0 || (a->raw && (b->raw || b->n == 0) && idx), "cmve_gt_thresholds: raw rows / idx missing");
  const float* aerr = mode_err(a, mode);
  CMVE_REQUIRE(aerr, "cmve_gt_thresholds: set has no error plane for this mode");
  dim3 grid((unsigned)((a->n_pad + 3) / 4)), block(256);
#define GT(TA, TB)                                                                                                   \
  hipLaunchKernelGGL((gt_thr_kernel<TA, TB>), grid, block, 0, h->stream, (const TA*)a->raw, a->raw_ld, a->inv_norm, \
                     aerr, a->n, a->n_pad, (const TB*)b->raw, b->raw_ld, b->inv_norm, b->err_max, a->d, a->d_pad,   \
                     mode, off, idx, sgt, thr_hi, thr_lo)
  if (a->raw_dtype == CMVE_F32 && b->raw_dtype == CMVE_F32) GT(float, float);
  else if (a->raw_dtype == CMVE_F32 && b->raw_dtype == CMVE_F64) GT(float, double);
  else if (a->raw_dtype == CMVE_F64 && b->raw_dtype == CMVE_F32) GT(double, float);
  else GT(double, double);
#undef GT
  return check_launch("gt_thr_kernel");
}

extern "C" int cmve_rank_from_matrix(cmve_handle_t h, const void* errors, int32_t dtype, int64_t n_rows,
                                     int64_t n_cols, int64_t ld, int32_t transposed, const int64_t* off,
                                     const int32_t* idx, int32_t* cnt) {
  CMVE_REQUIRE(h && errors && off && idx && cnt, "cmve_rank_from_matrix: NULL argument");
  CMVE_REQUIRE(n_rows >= 0 && n_cols >= 0 && ld >= n_cols, "cmve_rank_from_matrix: bad shape");
  CMVE_REQUIRE(dtype == CMVE_F32 || dtype == CMVE_F64, "cmve_rank_from_matrix: dtype must be F32/F64");
  if (n_rows == 0 || n_cols == 0) return CMVE_OK;
  if (!transposed) {
    if (dtype == CMVE_F32)
      hipLaunchKernelGGL(rank_rows_kernel<float>, dim3((unsigned)n_rows), dim3(256), 0, h->stream,
                         (const float*)errors, n_cols, ld, off, idx, cnt);
    else
      hipLaunchKernelGGL(rank_rows_kernel<double>, dim3((unsigned)n_rows), dim3(256), 0, h->stream,
                         (const double*)errors, n_cols, ld, off, idx, cnt);
  } else {
    CMVE_HIP(hipMemsetAsync(cnt, 0, sizeof(int32_t) * n_cols, h->stream));
    const int64_t splits = std::min<int64_t>(64, (n_rows + 255) / 256);
    const int64_t rps = (n_rows + splits - 1) / splits;
    dim3 grid((unsigned)((n_cols + 255) / 256), (unsigned)splits);
    if (dtype == CMVE_F32)
      hipLaunchKernelGGL(rank_cols_kernel<float>, grid, dim3(256), 0, h->stream, (const float*)errors, n_rows, n_cols,
                         ld, rps, off, idx, cnt);
    else
      hipLaunchKernelGGL(rank_cols_kernel<double>, grid, dim3(256), 0, h->stream, (const double*)errors, n_rows,
                         n_cols, ld, rps, off, idx, cnt);
  }
  return check_launch("rank_from_matrix");
}

extern "C" int cmve_gt_positions_from_matrix(cmve_handle_t h, const void* errors, int32_t dtype, int64_t n_rows,
                                             int64_t n_cols, int64_t ld, int32_t transposed, const int64_t* off,
                                             const int32_t* idx, int32_t* pos) {
  CMVE_REQUIRE(h && errors && off && idx && pos, "cmve_gt_positions_from_matrix: NULL argument");
  CMVE_REQUIRE(n_rows >= 0 && n_cols >= 0 && ld >= n_cols, "cmve_gt_positions_from_matrix: bad shape");
  CMVE_REQUIRE(dtype == CMVE_F32 || dtype == CMVE_F64, "cmve_gt_positions_from_matrix: dtype must be F32/F64");
  if (n_rows == 0 || n_cols == 0) return CMVE_OK;
  if (!transposed) {
    if (dtype == CMVE_F32)
      hipLaunchKernelGGL(gtpos_rows_kernel<float>, dim3((unsigned)n_rows), dim3(256), 0, h->stream,
                         (const float*)errors, n_cols, ld, off, idx, pos);
    else
      hipLaunchKernelGGL(gtpos_rows_kernel<double>, dim3((unsigned)n_rows), dim3(256), 0, h->stream,
                         (const double*)errors, n_cols, ld, off, idx, pos);
  } else {
    dim3 grid((unsigned)((n_cols + 63) / 64));
    if (dtype == CMVE_F32)
      hipLaunchKernelGGL(gtpos_cols_kernel<float>, grid, dim3(256), 0, h->stream, (const float*)errors, n_rows,
                         n_cols, ld, off, idx, pos);
    else
      hipLaunchKernelGGL(gtpos_cols_kernel<double>, grid, dim3(256), 0, h->stream, (const double*)errors, n_rows,
                         n_cols, ld, off, idx, pos);
  }
  return check_launch("gt_positions_from_matrix");
}

extern "C" int cmve_rank_thresholds(cmve_handle_t h, const cmve_rows_t* a, const cmve_rows_t* b, int32_t mode,
                                    const double* sgt, float* thr_hi, float* thr_lo) {
  CMVE_REQUIRE(h && a && b && sgt && thr_hi && thr_lo, "cmve_rank_thresholds: NULL argument");
  CMVE_REQUIRE(a->d_pad == b->d_pad, "cmve_rank_thresholds: dimension mismatch");
  CMVE_REQUIRE(!((a->flags | b->flags) & CMVE_PACK_RAW), "cmve_rank_thresholds: sets packed CMVE_PACK_RAW have no score bound");
  CMVE_REQUIRE(mode == CMVE_SIM_BF16 || mode == CMVE_SIM_BF16X3 || mode == CMVE_SIM_F16,
               "cmve_rank_thresholds: unknown mode");
  const float* aerr = mode_err(a, mode);
  CMVE_REQUIRE(aerr, "cmve_rank_thresholds: set has no error plane for this mode");
  hipLaunchKernelGGL(thr_from_sgt_kernel, dim3((unsigned)((a->n_pad + 255) / 256)), dim3(256), 0, h->stream, sgt, aerr,
                     a->n, a->n_pad, b->err_max, a->d_pad, mode, thr_hi, thr_lo);
  return check_launch("thr_from_sgt_kernel");
}
