// K4(c) + K5: exact top-k per query -- LINAS-engine/inference.py:78-79
// (errors = cal_error(video_embs, cap_emb); np.argsort(errors[0])[:topK]).
//
// 1. approximate scores s~ [n_q, n_g] fp32 into the workspace:
//      n_q <= 32 : K12a gemv_scores_kernel -- the gallery streamed ONCE from HBM (the fp16 plane,
//                  2 B per element), 16 gallery rows per wave per MFMA, the (<= 32) query rows
//                  staged in LDS as the A operand: the inference.py regime (one caption against
//                  the whole gallery) is an HBM-bound GEMV, not a 256-row GEMM tile
//      otherwise : K4 sim_store (the G128 / G256 MFMA GEMM)
// 2. K12b score_hist_kernel: per query a 4096-bin histogram of s~ over [-1, 1] (bin width
//    2^-11), many blocks per query;
// 3. K12c topk_thresh_kernel: the bin b* holding the k-th largest s~ gives a lower bound
//    L <= T~_k; tau = round_down(L - 2E) (E = rigorous score error bound, DESIGN.md s4:
//    every true top-k column has s~ >= T~_k - 2E >= tau);
// 4. K12d topk_collect_kernel: columns with s~ >= tau -> a per-query candidate list;
// 5. K12e topk_finish_kernel: one block per query -- radix select of T~_k over the candidates,
//    band s~ >= T~_k - 2E, exact fp64 re-score (cos64, the rank path's routine), LDS bitonic
//    sort (score desc, index asc).  A query whose candidate list overflowed selects over its
//    dense workspace row instead (same code, dense source): exact either way.
// The score matrix is read twice by many blocks per query (histogram, collect) instead of
// five times by one block per query (the 4-pass radix select of the first version).
#include "cmve_internal.h"

namespace cmve {

typedef _Float16 tk_f16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 tk_bf16x8_t __attribute__((ext_vector_type(8)));
typedef short tk_s16x8_t __attribute__((ext_vector_type(8)));
typedef float tk_f32x4_t __attribute__((ext_vector_type(4)));

constexpr int TOPK_THREADS = 1024;
constexpr int TOPK_CAP = 4096;   // band columns re-scored per query (LDS: 4096 x 12 B)
constexpr int CAND_CAP = 8192;   // candidates per query from the histogram threshold (LDS: 8192 x 8 B)
constexpr int HBINS = 4096;      // histogram bins over [-1, 1]
constexpr int GEMV_MAX_Q = 32;   // K12a handles up to two 16-row query tiles
constexpr int GEMV_U = 8;        // k-steps (32 deep each) whose loads are issued together
constexpr int64_t CHUNK_MIN = 16384;  // histogram / collect columns per block (at least)

__device__ __forceinline__ uint32_t okey(float f) { return topk_key(f); }
__device__ __forceinline__ float okey_inv(uint32_t k) { return topk_key_inv(k); }
// monotone non-decreasing bin of a finite-or-infinite score (NaN excluded by the callers)
__device__ __forceinline__ int score_bin(float s) {
  const float t = fminf(fmaxf((s + 1.0f) * 2048.0f, 0.0f), (float)(HBINS - 1));
  return (int)t;
}

// ---------------------------------------------------------------------------
// K12a: small-batch scores.  Wave w of block b owns gallery rows [16 (4b + w), +16) (grid-stride);
// per 32-deep k-step a lane loads 16 B of one gallery row (row = lane & 15, k-chunk = lane >> 4:
// the B operand of v_mfma_f32_16x16x32) and reads the matching A fragment of each query tile from
// LDS, stored lane-linear per k-step (conflict-free ds_read_b128).  GEMV_U k-steps of loads are
// issued before their MFMAs; with ~16 waves per CU that keeps ~128 KiB in flight per CU.
// ---------------------------------------------------------------------------
template <int MODE>
__device__ __forceinline__ tk_f32x4_t tk_mfma(tk_s16x8_t a, tk_s16x8_t b, tk_f32x4_t c) {
  if constexpr (MODE == CMVE_SIM_F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(tk_f16x8_t, a), __builtin_bit_cast(tk_f16x8_t, b),
                                                  c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(tk_bf16x8_t, a),
                                                   __builtin_bit_cast(tk_bf16x8_t, b), c, 0, 0, 0);
}

template <int MODE, int NQT>
__global__ __launch_bounds__(256) void gemv_scores_kernel(const uint16_t* __restrict__ qhi,
                                                          const uint16_t* __restrict__ qlo,
                                                          const uint16_t* __restrict__ ghi,
                                                          const uint16_t* __restrict__ glo, int64_t d_pad, int nq,
                                                          int64_t ng, float* __restrict__ ws, int64_t ldw) {
  constexpr int PL = (MODE == CMVE_SIM_BF16X3) ? 2 : 1;  // planes: hi (+ lo)
  extern __shared__ tk_s16x8_t qa[];                      // [NQT][PL][nks][64] lane-linear fragments
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nks = (int)(d_pad >> 5);  // 32-deep k-steps
  // stage the query tiles: fragment (t, p, s, l) = plane p, row 16t + (l & 15), chunk 4s + (l >> 4)
  const int nfrag = NQT * PL * nks * 64;
  for (int f = tid; f < nfrag; f += 256) {
    const int l = f & 63, s = (f >> 6) % nks, tp = (f >> 6) / nks, p = tp % PL, t = tp / PL;
    const uint16_t* src = (p == 0 ? qhi : qlo) + (int64_t)(16 * t + (l & 15)) * d_pad + (4 * s + (l >> 4)) * 8;
    qa[f] = *(const tk_s16x8_t*)src;
  }
  __syncthreads();
  const int64_t ngroups = (ng + 15) >> 4;
  for (int64_t grp = (int64_t)blockIdx.x * 4 + wave; grp < ngroups; grp += (int64_t)gridDim.x * 4) {
    const int64_t row = grp * 16 + (lane & 15);  // < n_pad (rows padded to 256)
    const uint16_t* gh = ghi + row * d_pad + (lane >> 4) * 8;
    const uint16_t* gl = (PL == 2) ? glo + row * d_pad + (lane >> 4) * 8 : nullptr;
    tk_f32x4_t acc[NQT];
#pragma unroll
    for (int t = 0; t < NQT; ++t) acc[t] = tk_f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < nks; s0 += GEMV_U) {
      tk_s16x8_t bh[GEMV_U], bl[GEMV_U];
#pragma unroll
      for (int u = 0; u < GEMV_U; ++u) {
        if (s0 + u < nks) {
          bh[u] = __builtin_nontemporal_load((const tk_s16x8_t*)(gh + (s0 + u) * 32));
          if constexpr (PL == 2) bl[u] = __builtin_nontemporal_load((const tk_s16x8_t*)(gl + (s0 + u) * 32));
        }
      }
#pragma unroll
      for (int u = 0; u < GEMV_U; ++u) {
        if (s0 + u < nks) {
#pragma unroll
          for (int t = 0; t < NQT; ++t) {
            const tk_s16x8_t ah = qa[((t * PL) * nks + s0 + u) * 64 + lane];
            acc[t] = tk_mfma<MODE>(ah, bh[u], acc[t]);
            if constexpr (PL == 2) {
              const tk_s16x8_t al = qa[((t * PL + 1) * nks + s0 + u) * 64 + lane];
              acc[t] = tk_mfma<MODE>(ah, bl[u], acc[t]);
              acc[t] = tk_mfma<MODE>(al, bh[u], acc[t]);
            }
          }
        }
      }
    }
    // C[q = 16t + 4 (lane >> 4) + r][j = grp*16 + (lane & 15)]
    if (row < ng) {
#pragma unroll
      for (int t = 0; t < NQT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qi = 16 * t + 4 * (lane >> 4) + r;
          if (qi < nq) ws[(int64_t)qi * ldw + row] = acc[t][r];
        }
    }
  }
}

// ---------------------------------------------------------------------------
// K12b: histogram of s~ per query.  grid (nchunk, nq); a block owns columns [c0, c1) of one row.
// nchunk == 1: the block writes every bin (no pre-zeroing); else nonzero bins are added atomically
// into a zeroed histogram.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void score_hist_kernel(const float* __restrict__ ws, int64_t ldw, int64_t ng,
                                                          int64_t chunk, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[HBINS];
  const int tid = threadIdx.x;
  const int64_t q = blockIdx.y;
  for (int b = tid; b < HBINS; b += 1024) h[b] = 0;
  __syncthreads();
  const int64_t c0 = (int64_t)blockIdx.x * chunk, c1 = min(ng, c0 + chunk);
  const float* s = ws + q * ldw;
  // chunk and ldw are multiples of 4 and ws is 16-B aligned: float4 body, scalar tail
  const int64_t v1 = c0 + ((c1 - c0) & ~(int64_t)3);
  for (int64_t j = c0 + 4 * (int64_t)tid; j < v1; j += 4 * 1024) {
    const float4 v = *(const float4*)(s + j);
    if (v.x == v.x) atomicAdd(&h[score_bin(v.x)], 1u);
    if (v.y == v.y) atomicAdd(&h[score_bin(v.y)], 1u);
    if (v.z == v.z) atomicAdd(&h[score_bin(v.z)], 1u);
    if (v.w == v.w) atomicAdd(&h[score_bin(v.w)], 1u);
  }
  for (int64_t j = v1 + tid; j < c1; j += 1024) {
    const float v = s[j];
    if (v == v) atomicAdd(&h[score_bin(v)], 1u);
  }
  __syncthreads();
  uint32_t* out = hist + q * HBINS;
  if (gridDim.x == 1) {
    for (int b = tid; b < HBINS; b += 1024) out[b] = h[b];
  } else {
    for (int b = tid; b < HBINS; b += 1024)
      if (h[b]) atomicAdd(&out[b], h[b]);
  }
}

// ---------------------------------------------------------------------------
// K12c: per query, the bin b* where the count from the top first reaches k; L = lower edge of
// b* minus 2^-20 (covers the fp32 rounding of the bin arithmetic), tau = round_down(L - 2E).
// Fewer than k finite scores: keep every column (tau = -inf, keepall = 1, NaN included).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void topk_thresh_kernel(const uint32_t* __restrict__ hist, int k,
                                                          const float* __restrict__ qerr,
                                                          const float* __restrict__ gerr_max, int slot,
                                                          int64_t d_pad, int mode, float* __restrict__ tau,
                                                          int32_t* __restrict__ keepall) {
  __shared__ uint32_t part[256];
  const int tid = threadIdx.x;
  const int64_t q = blockIdx.x;
  const uint32_t* h = hist + q * HBINS;
  // thread t owns bins [HBINS - 16 (t+1), HBINS - 16 t): thread 0 the top of the range
  const int top = HBINS - 16 * tid;
  uint32_t mine = 0;
  for (int b = top - 16; b < top; ++b) mine += h[b];
  part[tid] = mine;
  __syncthreads();
  // inclusive scan (top first), Hillis-Steele in LDS
  for (int o = 1; o < 256; o <<= 1) {
    const uint32_t v = tid >= o ? part[tid - o] : 0u;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  const uint32_t total = part[255];
  const uint32_t before = tid ? part[tid - 1] : 0u;
  if (tid == 0 && total < (uint32_t)k) {
    tau[q] = -INFINITY;
    keepall[q] = 1;
  }
  if (total >= (uint32_t)k && before < (uint32_t)k && before + mine >= (uint32_t)k) {
    uint32_t acc = before;
    int b = top - 1;
    for (; b > top - 16; --b) {
      acc += h[b];
      if (acc >= (uint32_t)k) break;
    }
    const double E = score_error_bound((double)qerr[q], (double)gerr_max[slot], d_pad, mode);
    const double L = (b == 0) ? -INFINITY : (double)b / 2048.0 - 1.0 - 0x1p-20;
    tau[q] = f32_round_down(L - 2.0 * E);
    keepall[q] = 0;
  }
}

// ---------------------------------------------------------------------------
// K12d: candidates s~ >= tau[q] -> cand[q][0, CAND_CAP) (the count may exceed the capacity:
// the finish kernel then selects over the dense row).  One global atomic per wave with a hit.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void topk_collect_kernel(const float* __restrict__ ws, int64_t ldw, int64_t ng,
                                                           int64_t chunk, const float* __restrict__ tau,
                                                           const int32_t* __restrict__ keepall,
                                                           uint32_t* __restrict__ cnt, int32_t* __restrict__ cand) {
  const int lane = threadIdx.x & 63;
  const int64_t q = blockIdx.y;
  const float t = tau[q];
  const bool all = keepall[q] != 0;
  const int64_t c0 = (int64_t)blockIdx.x * chunk, c1 = min(ng, c0 + chunk);
  const float* s = ws + q * ldw;
  int32_t* cq = cand + q * CAND_CAP;
  for (int64_t jb = c0 + (threadIdx.x & ~63); jb < c1; jb += 256) {
    const int64_t j = jb + lane;
    const bool keep = j < c1 && (all || s[j] >= t);
    const uint64_t m = __ballot(keep);
    if (m == 0) continue;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&cnt[q], (uint32_t)__popcll(m));
    base = __shfl(base, 0, 64);
    if (keep) {
      const uint32_t p = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      if (p < (uint32_t)CAND_CAP) cq[p] = (int32_t)j;
    }
  }
}

// ---------------------------------------------------------------------------
// K12e (and the dense fallback): select the k-th largest s~ over a source of (score, column)
// entries, keep the 2E band, re-score it in fp64, sort, write the first k.
// ---------------------------------------------------------------------------
struct DenseSrc {  // one workspace row
  const float* s;
  int64_t n;
  __device__ float score(int64_t c) const { return s[c]; }
  __device__ int32_t col(int64_t c) const { return (int32_t)c; }
};
struct ListSrc {  // candidates staged in LDS
  const float* s;
  const int32_t* idx;
  int64_t n;
  __device__ float score(int64_t c) const { return s[c]; }
  __device__ int32_t col(int64_t c) const { return idx[c]; }
};

struct FinishLds {
  uint32_t hist[256];
  uint32_t sh_prefix, sh_need, sh_count;
  double cs[TOPK_CAP];
  int32_t ci[TOPK_CAP];
};

template <class Src, typename TQ, typename TG>
__device__ void select_rescore_sort(const Src& src, FinishLds& L, int64_t row, int k, const TQ* __restrict__ xq,
                                    const double qinv, const float qerr, const TG* __restrict__ graw, int64_t ldg,
                                    const double* __restrict__ ginv, const float gerr_max, int64_t d, int64_t d_pad,
                                    int mode, int32_t* __restrict__ out_idx, double* __restrict__ out_score,
                                    int32_t* __restrict__ overflow) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // ---- radix select of the k-th largest key (8-bit digits, 4 passes) ----
  uint32_t prefix = 0, mask = 0, need = (uint32_t)k;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int b = tid; b < 256; b += TOPK_THREADS) L.hist[b] = 0;
    __syncthreads();
    for (int64_t c = tid; c < src.n; c += TOPK_THREADS) {
      const uint32_t key = okey(src.score(c));
      if ((key & mask) == prefix) atomicAdd(&L.hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (wave == 0) {
      // digit holding the need-th largest key: bins from the top, 4 per lane, wave suffix sums
      // (a serial 256-bin walk by one thread was ~7 us of dependent LDS reads per pass)
      uint32_t hb[4], v = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) v += (hb[i] = L.hist[4 * lane + i]);
      uint32_t t = v;  // inclusive suffix sum over lanes >= lane
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_down(t, off, 64);
        if (lane + off < 64) t += o;
      }
      const uint32_t above = t - v;  // keys in bins above this lane's four
      const uint32_t total = __shfl(t, 0, 64);
      if (total < need) {  // fewer keys than needed: digit 0 (as the serial walk ends)
        if (lane == 0) {
          L.sh_prefix = prefix;
          L.sh_need = need - (total - hb[0]);
        }
      } else if (above < need && need <= t) {
        uint32_t acc = above;
        int b = 3;
        for (; b > 0; --b) {
          if (acc + hb[b] >= need) break;
          acc += hb[b];
        }
        L.sh_prefix = prefix | ((uint32_t)(4 * lane + b) << shift);
        L.sh_need = need - acc;
      }
    }
    __syncthreads();
    prefix = L.sh_prefix;
    need = L.sh_need;
    mask |= 255u << shift;
    __syncthreads();
  }
  // prefix is now the key of the k-th largest score (0: fewer than k finite scores)
  const uint32_t kk = prefix;
  const double E = score_error_bound((double)qerr, (double)gerr_max, d_pad, mode);
  const float tau = (kk == 0u) ? -INFINITY : f32_round_down((double)okey_inv(kk) - 2.0 * E);

  // ---- collect the band ----
  if (tid == 0) L.sh_count = 0;
  __syncthreads();
  for (int64_t c = tid; c < src.n; c += TOPK_THREADS) {
    const float v = src.score(c);
    if (v >= tau || (kk == 0u)) {  // kk == 0: keep everything
      const uint32_t p = atomicAdd(&L.sh_count, 1u);
      if (p < (uint32_t)TOPK_CAP) L.ci[p] = src.col(c);
    }
  }
  __syncthreads();
  const uint32_t cnt_all = L.sh_count;
  if (cnt_all > (uint32_t)TOPK_CAP && tid == 0) atomicOr(overflow, 1);
  const int cnt = (int)min(cnt_all, (uint32_t)TOPK_CAP);

  // ---- exact fp64 re-score (one wave per kept column) ----
  for (int c = wave; c < cnt; c += TOPK_THREADS / 64) {
    const int32_t j = L.ci[c];
    const double v = wave_dot64(xq, graw + (int64_t)j * ldg, d, lane) * (qinv * ginv[j]);
    if (lane == 0) L.cs[c] = (v == v) ? v : -INFINITY;
  }
  int npow = 1;
  while (npow < cnt) npow <<= 1;
  for (int c = cnt + tid; c < npow; c += TOPK_THREADS) {
    L.cs[c] = -INFINITY;
    L.ci[c] = 0x7fffffff;
  }
  __syncthreads();

  // ---- bitonic sort: descending score, ascending index ----
  for (int size = 2; size <= npow; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < npow / 2; t += TOPK_THREADS) {
        const int lo = 2 * stride * (t / stride) + (t % stride);
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);
        const double a = L.cs[lo], b = L.cs[hi];
        const int32_t ia = L.ci[lo], ib = L.ci[hi];
        const bool a_first = (a > b) || (a == b && ia < ib);  // "a before b" in the final order
        if (a_first != desc) {
          L.cs[lo] = b;
          L.cs[hi] = a;
          L.ci[lo] = ib;
          L.ci[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  for (int t = tid; t < k; t += TOPK_THREADS) {
    const bool ok = t < cnt;
    out_idx[row * k + t] = ok ? L.ci[t] : -1;
    out_score[row * k + t] = ok ? L.cs[t] : NAN;
  }
}

template <typename TQ, typename TG>
__global__ __launch_bounds__(TOPK_THREADS) void topk_finish_kernel(
    const float* __restrict__ ws, int64_t ldw, int64_t ng, int k, const uint32_t* __restrict__ cnt,
    const int32_t* __restrict__ cand, const TQ* __restrict__ qraw, int64_t ldq, const double* __restrict__ qinv,
    const float* __restrict__ qerr, const TG* __restrict__ graw, int64_t ldg, const double* __restrict__ ginv,
    const float* __restrict__ gerr_max, int slot, int64_t d, int64_t d_pad, int mode, int64_t list_cap,
    int32_t* __restrict__ out_idx, double* __restrict__ out_score, int32_t* __restrict__ overflow) {
  __shared__ FinishLds L;
  __shared__ float ls[CAND_CAP];
  __shared__ int32_t li[CAND_CAP];
  const int64_t row = blockIdx.x;
  const float* s = ws + row * ldw;
  const uint32_t n = cnt[row];
  const TQ* xq = qraw + row * ldq;
  if ((int64_t)n <= list_cap) {
    const int32_t* cq = cand + row * CAND_CAP;
    for (int c = threadIdx.x; c < (int)n; c += TOPK_THREADS) {
      const int32_t j = cq[c];
      li[c] = j;
      ls[c] = s[j];
    }
    __syncthreads();
    select_rescore_sort(ListSrc{ls, li, (int64_t)n}, L, row, k, xq, qinv[row], qerr[row], graw, ldg, ginv,
                        gerr_max[slot], d, d_pad, mode, out_idx, out_score, overflow);
  } else {
    select_rescore_sort(DenseSrc{s, ng}, L, row, k, xq, qinv[row], qerr[row], graw, ldg, ginv, gerr_max[slot], d,
                        d_pad, mode, out_idx, out_score, overflow);
  }
}

// workspace layout (in 4-byte units, sections 256-B aligned) for n_q queries over a gallery of n_pad rows
struct TopkWs {
  int64_t scores, hist, tau, keepall, cnt, cand, total;
};
static inline int64_t al64(int64_t x) { return (x + 63) & ~(int64_t)63; }
static TopkWs topk_ws_layout(int64_t nq, int64_t g_n_pad) {
  TopkWs w;
  w.scores = 0;
  w.hist = al64(nq * g_n_pad);
  w.tau = w.hist + al64(nq * HBINS);
  w.keepall = w.tau + al64(nq);
  w.cnt = w.keepall + al64(nq);
  w.cand = w.cnt + al64(nq);
  w.total = w.cand + al64(nq * CAND_CAP);
  return w;
}

template <int MODE>
static int launch_gemv(const cmve_rows_t* q, const cmve_rows_t* g, float* ws, hipStream_t stream) {
  constexpr int PL = (MODE == CMVE_SIM_BF16X3) ? 2 : 1;
  const uint16_t* qh = MODE == CMVE_SIM_F16 ? q->h16 : q->hi;
  const uint16_t* gh = MODE == CMVE_SIM_F16 ? g->h16 : g->hi;
  const int nqt = q->n <= 16 ? 1 : 2;
  const size_t lds = (size_t)nqt * PL * 16 * g->d_pad * 2;
  const int cus = device_cus();
  const int64_t groups = (g->n + 15) / 16;
  // enough blocks for ~16 waves per CU, never more than one 16-row group per wave
  const unsigned nblocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((groups + 3) / 4, (int64_t)cus * 4));
#define GV(NQT)                                                                                                     \
  do {                                                                                                              \
    static const hipError_t attr_err = hipFuncSetAttribute((const void*)gemv_scores_kernel<MODE, NQT>,              \
                                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
    CMVE_HIP(attr_err);                                                                                             \
    hipLaunchKernelGGL((gemv_scores_kernel<MODE, NQT>), dim3(nblocks), dim3(256), lds, stream, qh, q->lo, gh, g->lo, \
                       g->d_pad, (int)q->n, g->n, ws, g->n_pad);                                                    \
  } while (0)
  if (nqt == 1) GV(1);
  else GV(2);
#undef GV
  return check_launch("gemv_scores_kernel");
}

// ---------------------------------------------------------------------------
// K13: large-batch top-k without the score matrix (the C5 regime: 16,384 captions x a 131,072-row
// shard).  tau_i comes from a gallery SAMPLE (its first n_s rows): the k-th largest s~ of a subset
// is <= the k-th largest over the whole gallery, so tau_i = round_down(L_i - 2E) (K12c on the
// sample's histogram) is a valid candidate threshold for the full gallery (top-k).
// The main GEMM (sim.hip EPI_TOPK) then emits every s~ >= tau_i as (key(s~), row & 255, col),
// bucketed by 256-row query tile; K13b turns each query's entries into its exact top-k.
// ---------------------------------------------------------------------------
constexpr int BT_Q = 16;       // queries per finish block (one wave each)
constexpr int BT_LCAP = 512;   // entries kept per query (more: the row is left to the dense path)
constexpr int BT_BAND = 256;   // band entries re-scored per query
constexpr int BT_KMAX = 32;    // k * n_g / BT_TARGET sample rows must stay <= n_g / 4 to pay off
constexpr int BT_TARGET = 128; // expected entries per query the sample size is chosen for

__global__ __launch_bounds__(256) void topk_batch_thr_kernel(const float* __restrict__ tau,
                                                             const int32_t* __restrict__ keepall, int64_t nq,
                                                             int64_t nq_pad, float* __restrict__ hi,
                                                             float* __restrict__ lo) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= nq_pad) return;
  const bool ok = r < nq && !keepall[r] && tau[r] > -INFINITY && tau[r] < INFINITY;
  hi[r] = ok ? INFINITY : __builtin_nanf("");  // NaN: the row emits nothing (left to the dense path)
  lo[r] = ok ? tau[r] : __builtin_nanf("");
}

struct BatchLds {
  uint32_t key[BT_Q][BT_LCAP];
  int32_t col[BT_Q][BT_LCAP];
  double bs[BT_Q][BT_BAND];
  uint32_t cnt[BT_Q];
  int32_t nband[BT_Q];
};

template <typename TQ, typename TG>
__global__ __launch_bounds__(1024) void topk_batch_finish_kernel(
    const unsigned long long* __restrict__ bucket_cnt, const unsigned long long* __restrict__ cand, int64_t cap_b,
    int64_t nq, int k, const int32_t* __restrict__ keepall, const TQ* __restrict__ qraw, int64_t ldq,
    const double* __restrict__ qinv, const float* __restrict__ qerr, const TG* __restrict__ graw, int64_t ldg,
    const double* __restrict__ ginv, const float* __restrict__ gerr_max, int slot, int64_t d, int64_t d_pad, int mode,
    int32_t* __restrict__ out_idx, double* __restrict__ out_score, int32_t* __restrict__ unresolved) {
  __shared__ BatchLds L;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // XCD-aware order: the 16 blocks reading one bucket run on one XCD (its entries stay in that L2)
  const int total = (int)gridDim.x, bid = (int)blockIdx.x;
  const int xcd = bid & 7, local = bid >> 3, qq = total >> 3, rr = total & 7;
  const int lb = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + local;
  const int64_t q0 = (int64_t)lb * BT_Q;
  const int64_t bucket = q0 >> 8;
  if (tid < BT_Q) L.cnt[tid] = 0;
  __syncthreads();
  const unsigned long long nb_all = bucket_cnt[bucket];
  const bool bucket_ovf = nb_all > (unsigned long long)cap_b;
  const int64_t ne = (int64_t)min(nb_all, (unsigned long long)cap_b);
  const unsigned long long* e = cand + bucket * cap_b;
  const uint32_t r_lo = (uint32_t)(q0 & 255);
  for (int64_t t = tid; t < ne; t += 1024) {
    const unsigned long long v = e[t];
    const uint32_t rl = (uint32_t)(v >> 24) & 255u;
    if (rl - r_lo < (uint32_t)BT_Q) {
      const uint32_t p = atomicAdd(&L.cnt[rl - r_lo], 1u);
      if (p < (uint32_t)BT_LCAP) {
        L.key[rl - r_lo][p] = (uint32_t)(v >> 32);
        L.col[rl - r_lo][p] = (int32_t)(v & 0xffffffu);
      }
    }
  }
  __syncthreads();
  const int64_t row = q0 + w;
  const uint32_t n_all = L.cnt[w];
  const int m = (int)min(n_all, (uint32_t)BT_LCAP);
  bool ok = row < nq && !bucket_ovf && !keepall[row] && n_all <= (uint32_t)BT_LCAP && m >= k;
  // pad to BT_LCAP, then a block-wide bitonic sort of every wave's (key, col) row, key descending
  for (int t = m + lane; t < BT_LCAP; t += 64) {
    L.key[w][t] = 0u;
    L.col[w][t] = 0x7fffffff;
  }
  __syncthreads();
  for (int size = 2; size <= BT_LCAP; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = lane; t < BT_LCAP / 2; t += 64) {
        const int lo = 2 * stride * (t / stride) + (t % stride), hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const uint32_t ka = L.key[w][lo], kb = L.key[w][hi];
        const int32_t ia = L.col[w][lo], ib = L.col[w][hi];
        const bool a_first = ka > kb || (ka == kb && ia < ib);
        if (a_first != desc) {
          L.key[w][lo] = kb;
          L.key[w][hi] = ka;
          L.col[w][lo] = ib;
          L.col[w][hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  // band: the sorted prefix with s~ >= round_down(T~_k - 2E); fp64 re-score (cos64, K5's routine)
  int nb = 0;
  if (ok) {
    const double E = score_error_bound((double)qerr[row], (double)gerr_max[slot], d_pad, mode);
    const float thr = f32_round_down((double)topk_key_inv(L.key[w][k - 1]) - 2.0 * E);
    const uint32_t kthr = topk_key(thr);
    for (int t0 = 0; t0 < m; t0 += 64) {
      const int t = t0 + lane;
      const bool in = t < m && L.key[w][t] >= kthr;
      nb += __popcll(__ballot(in));
    }
    if (nb > BT_BAND) ok = false;
  }
  if (ok) {
    const TQ* xq = qraw + row * ldq;
    const double qi = qinv[row];
    for (int t = 0; t < nb; ++t) {
      const int32_t j = L.col[w][t];
      const double v = wave_dot64(xq, graw + (int64_t)j * ldg, d, lane) * (qi * ginv[j]);
      if (lane == 0) L.bs[w][t] = (v == v) ? v : -INFINITY;
    }
  } else {
    nb = 0;
  }
  for (int t = nb + lane; t < BT_BAND; t += 64) {
    L.bs[w][t] = -INFINITY;
    L.col[w][t] = 0x7fffffff;
  }
  __syncthreads();
  // band sort: fp64 score descending, column ascending (the dense path's order)
  for (int size = 2; size <= BT_BAND; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = lane; t < BT_BAND / 2; t += 64) {
        const int lo = 2 * stride * (t / stride) + (t % stride), hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const double a = L.bs[w][lo], b = L.bs[w][hi];
        const int32_t ia = L.col[w][lo], ib = L.col[w][hi];
        const bool a_first = a > b || (a == b && ia < ib);
        if (a_first != desc) {
          L.bs[w][lo] = b;
          L.bs[w][hi] = a;
          L.col[w][lo] = ib;
          L.col[w][hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  if (row < nq) {
    for (int t = lane; t < k; t += 64) {
      out_idx[row * k + t] = ok ? L.col[w][t] : -2;  // -2: unresolved, the caller's dense pass
      out_score[row * k + t] = ok ? L.bs[w][t] : NAN;
    }
    if (!ok && lane == 0) atomicAdd(unresolved, 1);
  }
}

// workspace of cmve_topk_batch (4-byte units, sections 256-B aligned)
struct BatchWs {
  int64_t ns, ns_pad, sc, hist, tau, keepall, hi, lo, cand, nb, cap_b, total;
};
static BatchWs batch_ws_layout(int64_t nq, int64_t nq_pad, int64_t g_n, int64_t g_n_pad, int k) {
  BatchWs w;
  const int64_t want = ((int64_t)k * g_n + BT_TARGET - 1) / BT_TARGET;
  w.ns = std::min<int64_t>(g_n, std::max<int64_t>(want, 2 * (int64_t)k));
  w.ns_pad = std::min<int64_t>(g_n_pad, (w.ns + 255) & ~(int64_t)255);
  w.sc = 0;
  w.hist = al64(nq * w.ns_pad);
  w.tau = w.hist + al64(nq * HBINS);
  w.keepall = w.tau + al64(nq);
  w.hi = w.keepall + al64(nq);
  w.lo = w.hi + al64(nq_pad);
  w.cand = w.lo + al64(nq_pad);
  w.nb = (nq_pad + 255) / 256;
  w.cap_b = 256 * (int64_t)BT_LCAP;
  w.total = w.cand + 2 * (w.nb + w.nb * w.cap_b);
  return w;
}

static bool gemv_fits(const cmve_rows_t* q, const cmve_rows_t* g, int mode) {
  const int nqt = q->n <= 16 ? 1 : 2;
  const size_t lds = (size_t)nqt * (mode == CMVE_SIM_BF16X3 ? 2 : 1) * 16 * g->d_pad * 2;
  return q->n <= GEMV_MAX_Q && lds <= 160 * 1024;
}

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_sim_store(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, float alpha,
                              float beta, void* out, int32_t out_dtype, int64_t ldo);

extern "C" int cmve_topk_workspace(const cmve_rows_t* q, const cmve_rows_t* g, int32_t k, int64_t* n_floats) {
  CMVE_REQUIRE(q && g && n_floats, "cmve_topk_workspace: NULL argument");
  CMVE_REQUIRE(k >= 1 && k <= TOPK_CAP / 2, "cmve_topk_workspace: k must be in [1, %d]", TOPK_CAP / 2);
  *n_floats = topk_ws_layout(std::max<int64_t>(q->n, 1), g->n_pad).total;
  return CMVE_OK;
}

extern "C" int cmve_topk(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, int32_t k,
                         float* scores_ws, int64_t ws_floats, int32_t* out_idx, double* out_score,
                         int32_t* overflow) {
  CMVE_REQUIRE(h && q && g && scores_ws && out_idx && out_score && overflow, "cmve_topk: NULL argument");
  CMVE_REQUIRE(k >= 1, "cmve_topk: k must be >= 1");
  CMVE_REQUIRE(k <= TOPK_CAP / 2, "cmve_topk: k must be <= %d", TOPK_CAP / 2);
  CMVE_REQUIRE(q->raw && g->raw && q->inv_norm && g->inv_norm, "cmve_topk: raw rows / norms missing");
  CMVE_REQUIRE(!((q->flags | g->flags) & CMVE_PACK_RAW), "cmve_topk: sets packed CMVE_PACK_RAW have no score bound");
  CMVE_REQUIRE(q->d == g->d && q->d_pad == g->d_pad && q->d_pad % 64 == 0, "cmve_topk: dimension mismatch");
  CMVE_REQUIRE(g->n < (1ll << 31), "cmve_topk: gallery too large for int32 indices");
  CMVE_REQUIRE(mode == CMVE_SIM_BF16 || mode == CMVE_SIM_BF16X3 || mode == CMVE_SIM_F16, "cmve_topk: unknown mode %d",
               mode);
  CMVE_HIP(hipMemsetAsync(overflow, 0, sizeof(int32_t), h->stream));
  if (q->n == 0) return CMVE_OK;
  const TopkWs w = topk_ws_layout(q->n, g->n_pad);
  CMVE_REQUIRE(ws_floats >= w.total, "cmve_topk: workspace has %lld floats, needs %lld (cmve_topk_workspace)",
               (long long)ws_floats, (long long)w.total);
  const float* qerr = mode_err(q, mode);
  CMVE_REQUIRE(qerr && g->err_max, "cmve_topk: set has no error plane for this mode");
  CMVE_REQUIRE(mode != CMVE_SIM_F16 || (q->h16 && g->h16), "cmve_topk: F16 needs h16 planes");
  CMVE_REQUIRE(mode != CMVE_SIM_BF16X3 || (q->lo && g->lo), "cmve_topk: BF16X3 needs lo planes");
  hipStream_t st = h->stream;
  float* scores = scores_ws + w.scores;
  uint32_t* hist = (uint32_t*)(scores_ws + w.hist);
  float* tau = scores_ws + w.tau;
  int32_t* keepall = (int32_t*)(scores_ws + w.keepall);
  uint32_t* cnt = (uint32_t*)(scores_ws + w.cnt);
  int32_t* cand = (int32_t*)(scores_ws + w.cand);
  if (g->n == 0) {
    CMVE_HIP(hipMemsetAsync(out_idx, 0xff, sizeof(int32_t) * q->n * k, st));
    return CMVE_OK;
  }

  // 1. approximate scores
  int rc;
  if (gemv_fits(q, g, mode)) {
    if (mode == CMVE_SIM_F16) rc = launch_gemv<CMVE_SIM_F16>(q, g, scores, st);
    else if (mode == CMVE_SIM_BF16) rc = launch_gemv<CMVE_SIM_BF16>(q, g, scores, st);
    else rc = launch_gemv<CMVE_SIM_BF16X3>(q, g, scores, st);
  } else {
    rc = cmve_sim_store(h, q, g, mode, 1.0f, 0.0f, scores, CMVE_F32, g->n_pad);
  }
  if (rc) return rc;

  // 2-4. histogram -> threshold -> candidates
  const int64_t want = std::max<int64_t>(1, 1024 / q->n);
  const int64_t max_chunks = std::max<int64_t>(1, (g->n + CHUNK_MIN - 1) / CHUNK_MIN);
  const int64_t nchunk = std::min(want, max_chunks);
  const int64_t chunk = (((g->n + nchunk - 1) / nchunk) + 255) & ~(int64_t)255;
  const int64_t nch = (g->n + chunk - 1) / chunk;
  if (nch > 1) CMVE_HIP(hipMemsetAsync(hist, 0, sizeof(uint32_t) * q->n * HBINS, st));
  CMVE_HIP(hipMemsetAsync(cnt, 0, sizeof(uint32_t) * q->n, st));
  hipLaunchKernelGGL(score_hist_kernel, dim3((unsigned)nch, (unsigned)q->n), dim3(1024), 0, st, scores, g->n_pad,
                     g->n, chunk, hist);
  rc = check_launch("score_hist_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(topk_thresh_kernel, dim3((unsigned)q->n), dim3(256), 0, st, hist, k, qerr, g->err_max,
                     mode_slot(mode), g->d_pad, mode, tau, keepall);
  rc = check_launch("topk_thresh_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(topk_collect_kernel, dim3((unsigned)nch, (unsigned)q->n), dim3(256), 0, st, scores, g->n_pad,
                     g->n, chunk, tau, keepall, cnt, cand);
  rc = check_launch("topk_collect_kernel");
  if (rc) return rc;

  // 5. select + exact re-score + sort.  A study build with -DCMVE_TOPK_DENSE=1 sends every query down the
  // dense-row path that a candidate-list overflow takes (tests reach it through near-duplicate galleries).
#ifndef CMVE_TOPK_DENSE
#define CMVE_TOPK_DENSE 0
#endif
  const int64_t list_cap = CMVE_TOPK_DENSE ? -1 : CAND_CAP;
#define TK(TQ, TG)                                                                                                 \
  hipLaunchKernelGGL((topk_finish_kernel<TQ, TG>), dim3((unsigned)q->n), dim3(TOPK_THREADS), 0, st, scores,       \
                     g->n_pad, g->n, k, cnt, cand, (const TQ*)q->raw, q->raw_ld, q->inv_norm, qerr,                \
                     (const TG*)g->raw, g->raw_ld, g->inv_norm, g->err_max, mode_slot(mode), q->d, q->d_pad, mode, \
                     list_cap, out_idx, out_score, overflow)
  if (q->raw_dtype == CMVE_F32 && g->raw_dtype == CMVE_F32) TK(float, float);
  else if (q->raw_dtype == CMVE_F32 && g->raw_dtype == CMVE_F64) TK(float, double);
  else if (q->raw_dtype == CMVE_F64 && g->raw_dtype == CMVE_F32) TK(double, float);
  else TK(double, double);
#undef TK
  return check_launch("topk_finish_kernel");
}

namespace cmve {
int launch_topk_gemm(hipStream_t s, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, const float* row_hi,
                     const float* row_lo, uint64_t* cand, int64_t nb, int64_t cap_b);
}

extern "C" int cmve_topk_batch_workspace(const cmve_rows_t* q, const cmve_rows_t* g, int32_t k, int64_t* sample_rows,
                                         int64_t* n_floats) {
  CMVE_REQUIRE(q && g && n_floats, "cmve_topk_batch_workspace: NULL argument");
  CMVE_REQUIRE(k >= 1 && k <= BT_KMAX, "cmve_topk_batch_workspace: k must be in [1, %d]", BT_KMAX);
  const BatchWs w = batch_ws_layout(std::max<int64_t>(q->n, 1), std::max<int64_t>(q->n_pad, 256), g->n, g->n_pad, k);
  *n_floats = w.total;
  if (sample_rows) *sample_rows = w.ns;
  return CMVE_OK;
}

extern "C" int cmve_topk_batch(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, int32_t k,
                               float* ws, int64_t ws_floats, int32_t* out_idx, double* out_score,
                               int32_t* unresolved) {
  CMVE_REQUIRE(h && q && g && ws && out_idx && out_score && unresolved, "cmve_topk_batch: NULL argument");
  CMVE_REQUIRE(k >= 1 && k <= BT_KMAX, "cmve_topk_batch: k must be in [1, %d]", BT_KMAX);
  CMVE_REQUIRE(q->raw && g->raw && q->inv_norm && g->inv_norm, "cmve_topk_batch: raw rows / norms missing");
  CMVE_REQUIRE(!((q->flags | g->flags) & CMVE_PACK_RAW), "cmve_topk_batch: sets packed CMVE_PACK_RAW have no score bound");
  CMVE_REQUIRE(q->d == g->d && q->d_pad == g->d_pad && q->d_pad % 64 == 0, "cmve_topk_batch: dimension mismatch");
  CMVE_REQUIRE(g->n < (1ll << 24), "cmve_topk_batch: gallery shard must hold < 2^24 rows");
  CMVE_REQUIRE(mode == CMVE_SIM_BF16 || mode == CMVE_SIM_BF16X3 || mode == CMVE_SIM_F16,
               "cmve_topk_batch: unknown mode %d", mode);
  CMVE_HIP(hipMemsetAsync(unresolved, 0, sizeof(int32_t), h->stream));
  if (q->n == 0) return CMVE_OK;
  hipStream_t st = h->stream;
  if (g->n == 0) {
    CMVE_HIP(hipMemsetAsync(out_idx, 0xff, sizeof(int32_t) * q->n * k, st));
    return CMVE_OK;
  }
  const BatchWs w = batch_ws_layout(q->n, q->n_pad, g->n, g->n_pad, k);
  CMVE_REQUIRE(ws_floats >= w.total, "cmve_topk_batch: workspace has %lld floats, needs %lld",
               (long long)ws_floats, (long long)w.total);
  const float* qerr = mode_err(q, mode);
  CMVE_REQUIRE(qerr && g->err_max, "cmve_topk_batch: set has no error plane for this mode");
  float* sc = ws + w.sc;
  uint32_t* hist = (uint32_t*)(ws + w.hist);
  float* tau = ws + w.tau;
  int32_t* keepall = (int32_t*)(ws + w.keepall);
  float* hi = ws + w.hi;
  float* lo = ws + w.lo;
  uint64_t* cand = (uint64_t*)(ws + w.cand);

  // 1. sample scores: the first ns gallery rows (a prefix view shares every plane and err_max)
  cmve_rows_t sv = *g;
  sv.n = w.ns;
  sv.n_pad = w.ns_pad;
  int rc = cmve_sim_store(h, q, &sv, mode, 1.0f, 0.0f, sc, CMVE_F32, w.ns_pad);
  if (rc) return rc;
  // 2. per-query tau from the sample's histogram (K12b / K12c)
  const int64_t nchunk = std::min<int64_t>(std::max<int64_t>(1, 1024 / q->n),
                                           std::max<int64_t>(1, (w.ns + CHUNK_MIN - 1) / CHUNK_MIN));
  const int64_t chunk = (((w.ns + nchunk - 1) / nchunk) + 255) & ~(int64_t)255;
  const int64_t nch = (w.ns + chunk - 1) / chunk;
  if (nch > 1) CMVE_HIP(hipMemsetAsync(hist, 0, sizeof(uint32_t) * q->n * HBINS, st));
  hipLaunchKernelGGL(score_hist_kernel, dim3((unsigned)nch, (unsigned)q->n), dim3(1024), 0, st, sc, w.ns_pad, w.ns,
                     chunk, hist);
  rc = check_launch("score_hist_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(topk_thresh_kernel, dim3((unsigned)q->n), dim3(256), 0, st, hist, k, qerr, g->err_max,
                     mode_slot(mode), g->d_pad, mode, tau, keepall);
  rc = check_launch("topk_thresh_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(topk_batch_thr_kernel, dim3((unsigned)((q->n_pad + 255) / 256)), dim3(256), 0, st, tau, keepall,
                     q->n, q->n_pad, hi, lo);
  rc = check_launch("topk_batch_thr_kernel");
  if (rc) return rc;
  // 3. the whole gallery: every s~ >= tau -> its query tile's bucket
  CMVE_HIP(hipMemsetAsync(cand, 0, sizeof(uint64_t) * w.nb, st));
  rc = launch_topk_gemm(st, q, g, mode, hi, lo, cand, w.nb, w.cap_b);
  if (rc) return rc;
  // 4. per query: select T~_k over its entries, fp64 re-score of the 2E band, sort
  const unsigned nblk = (unsigned)((q->n + BT_Q - 1) / BT_Q);
#define TB(TQ, TG)                                                                                                 \
  hipLaunchKernelGGL((topk_batch_finish_kernel<TQ, TG>), dim3(nblk), dim3(1024), 0, st,                           \
                     (const unsigned long long*)cand, (const unsigned long long*)(cand + w.nb), w.cap_b, q->n, k,  \
                     keepall, (const TQ*)q->raw, q->raw_ld, q->inv_norm, qerr, (const TG*)g->raw, g->raw_ld,      \
                     g->inv_norm, g->err_max, mode_slot(mode), q->d, q->d_pad, mode, out_idx, out_score, unresolved)
  if (q->raw_dtype == CMVE_F32 && g->raw_dtype == CMVE_F32) TB(float, float);
  else if (q->raw_dtype == CMVE_F32 && g->raw_dtype == CMVE_F64) TB(float, double);
  else if (q->raw_dtype == CMVE_F64 && g->raw_dtype == CMVE_F32) TB(double, float);
  else TB(double, double);
#undef TB
  return check_launch("topk_batch_finish_kernel");
}

// ---------------------------------------------------------------------------
// K12f: the exact dense top-k of topk's band-overflow fallback (engine._topk_dense_exact): per query row,
// the k best of [its running best (kb entries, global ids) | a chunk of fp64 scores (ids j0 + c)] by (score
// desc, id asc) -- the order of np.argsort on the errors with NaN last (NaN scores count as -inf, as the
// caller's nan_to_num, and -0.0 as +0.0).  One block per row: an MSD radix select on the 64-bit
// order-preserving score key finds the k-th largest key T and how many entries equal to T enter, a second
// radix select on the ids among the keys == T picks the smallest of those ids, and the k winners are
// bitonic-sorted in LDS.  A rare path (near-duplicate gallery rows): ~13 passes over the row from L2.
// ---------------------------------------------------------------------------
constexpr int TD_THREADS = 256;
constexpr int TD_KMAX = 2048;

__device__ __forceinline__ uint64_t td_key(double s) {  // larger score -> larger key
  if (s != s) s = -INFINITY;
  if (s == 0.0) s = 0.0;  // -0.0 ties +0.0, as the comparison sort
  const uint64_t u = (uint64_t)__double_as_longlong(s);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

__global__ __launch_bounds__(TD_THREADS) void topk_dense_kernel(const double* __restrict__ best_s,
                                                                const int64_t* __restrict__ best_i, int64_t kb,
                                                                const double* __restrict__ s, int64_t lds,
                                                                int64_t nc, int64_t j0, int k,
                                                                double* __restrict__ out_s,
                                                                int64_t* __restrict__ out_i) {
  __shared__ uint32_t hist[256];
  __shared__ uint64_t s_prefix;
  __shared__ uint32_t s_want;
  __shared__ uint32_t n_sel;
  __shared__ uint64_t wk[TD_KMAX];
  __shared__ int64_t wi[TD_KMAX];
  const int64_t row = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t N = kb + nc;
  const int keff = (int)(N < k ? N : k);
  auto cand = [&](int64_t c, uint64_t& key, int64_t& id) {
    if (c < kb) {
      key = td_key(best_s[row * kb + c]);
      id = best_i[row * kb + c];
    } else {
      key = td_key(s[row * lds + (c - kb)]);
      id = j0 + (c - kb);
    }
  };
  // radix-select the keff-th largest key: `want` = its rank among the keys matching the prefix so far
  if (tid == 0) {
    s_prefix = 0ull;
    s_want = (uint32_t)keff;
  }
  uint64_t mask = 0ull;
  for (int shift = 56; shift >= 0 && keff < N && keff > 0; shift -= 8) {
    for (int b = tid; b < 256; b += TD_THREADS) hist[b] = 0u;
    __syncthreads();
    const uint64_t prefix = s_prefix;
    for (int64_t c = tid; c < N; c += TD_THREADS) {
      uint64_t key;
      int64_t id;
      cand(c, key, id);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t want = s_want, acc = 0u;
      int dgt = 255;
      while (acc + hist[dgt] < want) acc += hist[dgt--];
      s_want = want - acc;
      s_prefix = prefix | ((uint64_t)dgt << shift);
    }
    mask |= 0xffull << shift;
    __syncthreads();
  }
  // T = s_prefix (all 64 bits fixed); take every key > T and the s_want smallest ids among the keys == T.
  // The tied ids are radix-selected (ascending) the same way: their s_want-th smallest id is idT.
  const bool all = keff >= N;
  const uint64_t T = s_prefix;
  __shared__ uint64_t s_idpre;
  __shared__ uint32_t s_idwant;
  if (tid == 0) {
    s_idpre = 0ull;
    s_idwant = s_want;
  }
  __syncthreads();
  uint64_t imask = 0ull;
  for (int shift = 56; shift >= 0 && !all && keff > 0; shift -= 8) {
    for (int b = tid; b < 256; b += TD_THREADS) hist[b] = 0u;
    __syncthreads();
    const uint64_t pre = s_idpre;
    for (int64_t c = tid; c < N; c += TD_THREADS) {
      uint64_t key;
      int64_t id;
      cand(c, key, id);
      if (key == T && (((uint64_t)id) & imask) == pre) atomicAdd(&hist[(((uint64_t)id) >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t want = s_idwant, acc = 0u;
      int dgt = 0;
      while (acc + hist[dgt] < want) acc += hist[dgt++];
      s_idwant = want - acc;
      s_idpre = pre | ((uint64_t)dgt << shift);
    }
    imask |= 0xffull << shift;
    __syncthreads();
  }
  const uint64_t idT = s_idpre;
  if (tid == 0) n_sel = 0u;
  __syncthreads();
  for (int64_t c = tid; c < N; c += TD_THREADS) {
    uint64_t key;
    int64_t id;
    cand(c, key, id);
    if (all || key > T || (key == T && (uint64_t)id <= idT)) {
      const uint32_t p = atomicAdd(&n_sel, 1u);
      if (p < (uint32_t)TD_KMAX) {
        wk[p] = key;
        wi[p] = id;
      }
    }
  }
  __syncthreads();
  int P = 1;
  while (P < keff) P <<= 1;
  for (int t = (int)n_sel + tid; t < P; t += TD_THREADS) {  // padding sorts last
    wk[t] = 0ull;
    wi[t] = INT64_MAX;
  }
  __syncthreads();
  // bitonic sort, "before" = (key desc, id asc)
  for (int size = 2; size <= P; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < P; t += TD_THREADS) {
        const int o = t ^ stride;
        if (o > t) {
          const bool up = (t & size) == 0;
          const bool before_o = wk[o] > wk[t] || (wk[o] == wk[t] && wi[o] < wi[t]);
          if (before_o == up) {
            const uint64_t k2 = wk[t];
            wk[t] = wk[o];
            wk[o] = k2;
            const int64_t i2 = wi[t];
            wi[t] = wi[o];
            wi[o] = i2;
          }
        }
      }
      __syncthreads();
    }
  for (int t = tid; t < k; t += TD_THREADS) {
    if (t < keff) {
      const uint64_t kk = wk[t];
      const uint64_t u = (kk & 0x8000000000000000ull) ? (kk & 0x7fffffffffffffffull) : ~kk;
      out_s[row * k + t] = __longlong_as_double((long long)u);
      out_i[row * k + t] = wi[t];
    } else {
      out_s[row * k + t] = -INFINITY;
      out_i[row * k + t] = -1;
    }
  }
}

extern "C" int cmve_topk_dense_merge(cmve_handle_t h, const double* best_s, const int64_t* best_i, int64_t kb,
                                     const double* scores, int64_t lds, int64_t n_rows, int64_t nc, int64_t j0,
                                     int32_t k, double* out_s, int64_t* out_i) {
  CMVE_REQUIRE(h && (kb == 0 || (best_s && best_i)) && (nc == 0 || scores) && out_s && out_i,
               "cmve_topk_dense_merge: NULL argument");
  CMVE_REQUIRE(k >= 1 && k <= TD_KMAX && kb >= 0 && kb <= k && nc >= 0 && n_rows >= 0 && lds >= nc && j0 >= 0,
               "cmve_topk_dense_merge: bad shape (1 <= k <= %d, 0 <= kb <= k)", TD_KMAX);
  CMVE_REQUIRE(kb + nc < (1ll << 32), "cmve_topk_dense_merge: more than 2^32 candidates per row");
  if (n_rows == 0) return CMVE_OK;
  CMVE_REQUIRE((const void*)out_s != (const void*)best_s && (const void*)out_i != (const void*)best_i,
               "cmve_topk_dense_merge: out must not alias the running best");
  hipLaunchKernelGGL(topk_dense_kernel, dim3((unsigned)n_rows), dim3(TD_THREADS), 0, h->stream, best_s, best_i, kb,
                     scores, lds, nc, j0, (int)k, out_s, out_i);
  return check_launch("topk_dense_kernel");
}
