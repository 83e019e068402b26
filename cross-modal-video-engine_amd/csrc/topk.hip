// K4(c) + K5: exact top-k per query -- LINAS-engine/inference.py:78-79
// (errors = cal_error(video_embs, cap_emb); np.argsort(errors[0])[:topK]).
//
// 1. sim_store (bf16 MFMA) writes approximate scores s~ into a workspace row.
// 2. one 1024-thread block per query: 4-pass radix select (8-bit digits on the
//    order-preserving uint image of the float) finds the k-th largest s~ (T_k); every
//    column with s~ >= T_k - 2E is kept (E = rigorous score error bound, so the true
//    top-k is a subset of the kept columns: |T~_k - T_k| <= E).
// 3. the kept columns are re-scored in fp64 (cos64, same routine as the rank path),
//    bitonic-sorted in LDS by (score desc, index asc) and the first k written out.
#include "cmve_internal.h"

namespace cmve {

constexpr int TOPK_THREADS = 1024;
constexpr int TOPK_CAP = 4096;  // kept columns per query (LDS: 4096 x 12 B)

__device__ __forceinline__ uint32_t okey(float f) {
  const uint32_t u = __float_as_uint(f);
  if (f != f) return 0u;  // NaN ranks last (np.argsort puts NaN errors last)
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <typename TQ, typename TG>
__global__ __launch_bounds__(TOPK_THREADS) void topk_kernel(const float* __restrict__ scores, int64_t lds_,
                                                            int64_t ng, int k, const TQ* __restrict__ qraw,
                                                            int64_t ldq, const double* __restrict__ qinv,
                                                            const float* __restrict__ qerr,
                                                            const TG* __restrict__ graw, int64_t ldg,
                                                            const double* __restrict__ ginv,
                                                            const float* __restrict__ gerr_max, int64_t d,
                                                            int64_t d_pad, int mode, int32_t* __restrict__ out_idx,
                                                            double* __restrict__ out_score,
                                                            int32_t* __restrict__ overflow) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t sh_prefix, sh_need, sh_count;
  __shared__ double cs[TOPK_CAP];
  __shared__ int32_t ci[TOPK_CAP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t row = blockIdx.x;
  const float* s = scores + row * lds_;

  // ---- radix select of the k-th largest key ----
  uint32_t prefix = 0, mask = 0, need = (uint32_t)k;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int b = tid; b < 256; b += TOPK_THREADS) hist[b] = 0;
    __syncthreads();
    for (int64_t j = tid; j < ng; j += TOPK_THREADS) {
      const uint32_t key = okey(s[j]);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t acc = 0;
      int b = 255;
      for (; b > 0; --b) {
        if (acc + hist[b] >= need) break;
        acc += hist[b];
      }
      sh_prefix = prefix | ((uint32_t)b << shift);
      sh_need = need - acc;
    }
    __syncthreads();
    prefix = sh_prefix;
    need = sh_need;
    mask |= 255u << shift;
    __syncthreads();
  }
  // prefix is now the key of the k-th largest score
  const uint32_t kk = prefix;
  const float tk = __uint_as_float((kk & 0x80000000u) ? (kk & 0x7fffffffu) : ~kk);
  const double E = score_error_bound((double)qerr[row], (double)gerr_max[mode_slot(mode)], d_pad, mode);
  const float tau = (kk == 0u) ? -INFINITY : f32_round_down((double)tk - 2.0 * E);

  // ---- collect the band ----
  if (tid == 0) sh_count = 0;
  __syncthreads();
  for (int64_t j = tid; j < ng; j += TOPK_THREADS) {
    const float v = s[j];
    if (v >= tau || (kk == 0u)) {  // kk == 0: fewer than k finite scores -> keep everything
      const uint32_t p = atomicAdd(&sh_count, 1u);
      if (p < (uint32_t)TOPK_CAP) ci[p] = (int32_t)j;
    }
  }
  __syncthreads();
  const uint32_t cnt_all = sh_count;
  if (cnt_all > (uint32_t)TOPK_CAP && tid == 0) atomicOr(overflow, 1);
  const int cnt = (int)min(cnt_all, (uint32_t)TOPK_CAP);

  // ---- exact fp64 re-score (one wave per kept column) ----
  const TQ* xq = qraw + row * ldq;
  for (int c = wave; c < cnt; c += TOPK_THREADS / 64) {
    const int32_t j = ci[c];
    double v = wave_dot64(xq, graw + (int64_t)j * ldg, d, lane) * (qinv[row] * ginv[j]);
    if (lane == 0) cs[c] = (v == v) ? v : -INFINITY;
  }
  int npow = 1;
  while (npow < cnt) npow <<= 1;
  for (int c = cnt + tid; c < npow; c += TOPK_THREADS) {
    cs[c] = -INFINITY;
    ci[c] = 0x7fffffff;
  }
  __syncthreads();

  // ---- bitonic sort: descending score, ascending index ----
  for (int size = 2; size <= npow; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < npow / 2; t += TOPK_THREADS) {
        const int lo = 2 * stride * (t / stride) + (t % stride);
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);
        const double a = cs[lo], b = cs[hi];
        const int32_t ia = ci[lo], ib = ci[hi];
        // "a before b" in final order
        const bool a_first = (a > b) || (a == b && ia < ib);
        if (a_first != desc) {
          cs[lo] = b;
          cs[hi] = a;
          ci[lo] = ib;
          ci[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  for (int t = tid; t < k; t += TOPK_THREADS) {
    const bool ok = t < cnt;
    out_idx[row * k + t] = ok ? ci[t] : -1;
    out_score[row * k + t] = ok ? cs[t] : NAN;
  }
}

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_sim_store(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, float alpha,
                              float beta, void* out, int32_t out_dtype, int64_t ldo);

extern "C" int cmve_topk(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, int32_t k,
                         float* scores_ws, int32_t* out_idx, double* out_score, int32_t* overflow) {
  CMVE_REQUIRE(h && q && g && scores_ws && out_idx && out_score && overflow, "cmve_topk: NULL argument");
  CMVE_REQUIRE(k >= 1, "cmve_topk: k must be >= 1");
  CMVE_REQUIRE(k <= TOPK_CAP / 2, "cmve_topk: k must be <= %d", TOPK_CAP / 2);
  CMVE_REQUIRE(q->raw && g->raw && q->inv_norm && g->inv_norm, "cmve_topk: raw rows / norms missing");
  CMVE_HIP(hipMemsetAsync(overflow, 0, sizeof(int32_t), h->stream));
  if (q->n == 0) return CMVE_OK;
  int st = cmve_sim_store(h, q, g, mode, 1.0f, 0.0f, scores_ws, CMVE_F32, g->n_pad);
  if (st) return st;
  const float* qerr = mode_err(q, mode);
  CMVE_REQUIRE(qerr, "cmve_topk: set has no error plane for this mode");
#define TK(TQ, TG)                                                                                                \
  hipLaunchKernelGGL((topk_kernel<TQ, TG>), dim3((unsigned)q->n), dim3(TOPK_THREADS), 0, h->stream, scores_ws,    \
                     g->n_pad, g->n, k, (const TQ*)q->raw, q->raw_ld, q->inv_norm, qerr, (const TG*)g->raw,       \
                     g->raw_ld, g->inv_norm, g->err_max, q->d, q->d_pad, mode, out_idx, out_score, overflow)
  if (q->raw_dtype == CMVE_F32 && g->raw_dtype == CMVE_F32) TK(float, float);
  else if (q->raw_dtype == CMVE_F32 && g->raw_dtype == CMVE_F64) TK(float, double);
  else if (q->raw_dtype == CMVE_F64 && g->raw_dtype == CMVE_F32) TK(double, float);
  else TK(double, double);
#undef TK
  return check_launch("topk_kernel");
}
