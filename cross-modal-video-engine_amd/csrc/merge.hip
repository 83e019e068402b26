// C3: k-way merge of per-shard exact top-k lists (the gallery sharded over the ranks).
//
// After the all-gather of every shard's local top-k (global ids, fp64 cosines), query i holds `lists`
// sorted runs of k_in entries (score desc, id asc; empty slots id < 0 at a run's tail).  One wave per
// query: lane l holds the head of run l, and each of the k_out steps picks the best head by
// (score desc, id asc) with a 6-step butterfly and advances that run.  The output order is the
// reference's np.argsort(errors[0])[:topK] (LINAS-engine/inference.py:79) on tie-free scores, ties
// broken by the lower global id (a stable sort of the unsharded gallery).  NaN scores (zero-norm rows:
// np.argsort puts NaN errors last) rank after every number.
#include "cmve_internal.h"

namespace cmve {

// a strictly better than b: score desc (NaN last), then id asc; an empty head (id < 0) is worst
__device__ __forceinline__ bool head_better(double sa, int64_t ia, double sb, int64_t ib) {
  if (ia < 0) return false;
  if (ib < 0) return true;
  const bool na = sa != sa, nb = sb != sb;
  if (na != nb) return nb;
  if (!na && sa != sb) return sa > sb;
  return ia < ib;
}

// entry (query q, run l, position p) at q * q_stride + l * l_stride + p: query-major runs side by side
// (q_stride = lists * k_in, l_stride = k_in) or the rank-major layout of an all-gather (q_stride = k_in,
// l_stride = n_q * k_in)
__global__ __launch_bounds__(256) void merge_topk_kernel(const int64_t* __restrict__ ids,
                                                         const double* __restrict__ scores, int64_t n_q, int lists,
                                                         int k_in, int64_t q_stride, int64_t l_stride, int k_out,
                                                         int64_t* __restrict__ out_ids,
                                                         double* __restrict__ out_scores) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= n_q) return;
  const int64_t run = q * q_stride + (int64_t)lane * l_stride;
  int pos = 0;
  int64_t hid = -1;
  double hs = 0.0;
  auto load_head = [&]() {
    hid = -1;
    if (lane < lists && pos < k_in) {
      hid = ids[run + pos];
      hs = scores[run + pos];
    }
  };
  load_head();
  for (int t = 0; t < k_out; ++t) {
    double bs = hs;
    int64_t bi = hid;
    int bl = lane;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const double s2 = __shfl_xor(bs, o, 64);
      const int64_t i2 = __shfl_xor(bi, o, 64);
      const int l2 = __shfl_xor(bl, o, 64);
      // (score, id) keys are distinct across valid heads; empty heads tie on lane for determinism
      if (head_better(s2, i2, bs, bi) || (i2 < 0 && bi < 0 && l2 < bl)) {
        bs = s2;
        bi = i2;
        bl = l2;
      }
    }
    if (lane == 0) {
      out_ids[q * k_out + t] = bi < 0 ? -1 : bi;
      out_scores[q * k_out + t] = bi < 0 ? (double)NAN : bs;
    }
    if (bi >= 0 && lane == bl) {
      ++pos;
      load_head();
    }
  }
}

int merge_topk_launch(hipStream_t s, const int64_t* ids, const double* scores, int64_t n_q, int lists, int k_in,
                      int64_t q_stride, int64_t l_stride, int k_out, int64_t* out_ids, double* out_scores) {
  if (n_q == 0) return CMVE_OK;
  hipLaunchKernelGGL(merge_topk_kernel, dim3((unsigned)((n_q + 3) / 4)), dim3(256), 0, s, ids, scores, n_q, lists,
                     k_in, q_stride, l_stride, k_out, out_ids, out_scores);
  return check_launch("merge_topk_kernel");
}

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_merge_topk(cmve_handle_t h, const int64_t* ids, const double* scores, int64_t n_q, int32_t lists,
                               int32_t k_in, int32_t k_out, int64_t* out_ids, double* out_scores) {
  CMVE_REQUIRE(h && ids && scores && out_ids && out_scores, "cmve_merge_topk: NULL argument");
  CMVE_REQUIRE(n_q >= 0 && lists >= 1 && lists <= 64 && k_in >= 1 && k_out >= 1,
               "cmve_merge_topk: need 1 <= lists <= 64, k_in >= 1, k_out >= 1");
  return merge_topk_launch(h->stream, ids, scores, n_q, (int)lists, (int)k_in, (int64_t)lists * k_in, k_in, (int)k_out,
                           out_ids, out_scores);
}
