// Gallery-shard collectives of SURVEY.md 8(e) in the C ABI (8(b): cmve_dist_init / allgather_q /
// reduce_rank / allgather_topk), for a host that shards the gallery without torch.distributed (the
// Python host mirror, cmve/dist.py, runs the same exchange over torch.distributed).
// Per batch (the reference never shards -- LINAS-engine/evaluation.py:17-21 scores one in-memory
// gallery): all-gather the query rows over xGMI, every rank scores its resident shard, then one
// all-reduce MAX of the per-shard best-GT scores and one all-reduce SUM of the better-than-GT counts;
// top-k runs are all-gathered and merged on the device.  RCCL is opened with dlopen at first use (no link
// dependency: libcmve.so loads without it, and inside a torch process the RCCL torch already mapped
// is reused, one RCCL per process).  Every collective is enqueued on the handle's stream.
#include <dlfcn.h>
#include <string.h>
#include <rccl/rccl.h>

#include "cmve_internal.h"

namespace cmve {

struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*);
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*comm_destroy)(ncclComm_t);
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
  const char* (*error_string)(ncclResult_t);
  bool ok = false;
};

static RcclApi load_rccl() {
  RcclApi api{};
  void* lib = nullptr;
  // the soname first: a process that already mapped an RCCL (torch's, soname librccl.so.1) gets THAT one
  // back instead of a second copy from the library path
  for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
    if ((lib = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
  if (!lib) return api;
  api.get_unique_id = (decltype(api.get_unique_id))dlsym(lib, "ncclGetUniqueId");
  api.comm_init_rank = (decltype(api.comm_init_rank))dlsym(lib, "ncclCommInitRank");
  api.comm_destroy = (decltype(api.comm_destroy))dlsym(lib, "ncclCommDestroy");
  api.all_gather = (decltype(api.all_gather))dlsym(lib, "ncclAllGather");
  api.all_reduce = (decltype(api.all_reduce))dlsym(lib, "ncclAllReduce");
  api.error_string = (decltype(api.error_string))dlsym(lib, "ncclGetErrorString");
  api.ok = api.get_unique_id && api.comm_init_rank && api.comm_destroy && api.all_gather && api.all_reduce &&
           api.error_string;
  return api;
}

static const RcclApi* rccl_api() {
  static const RcclApi api = load_rccl();  // C++11 function-local static: initialised once, thread-safe
  return api.ok ? &api : nullptr;
}

#define CMVE_RCCL(api, call, what)                                                         \
  do {                                                                                     \
    const ncclResult_t r_ = (call);                                                        \
    if (r_ != ncclSuccess) {                                                               \
      ::cmve::set_error("%s: RCCL error %d: %s", what, (int)r_, (api)->error_string(r_));   \
      return CMVE_E_HIP;                                                                   \
    }                                                                                      \
  } while (0)

void dist_release(cmve_handle* h) {
  if (!h->comm) return;  // (no dlopen for handles that never held a communicator)
  const RcclApi* api = rccl_api();
  if (api) (void)api->comm_destroy((ncclComm_t)h->comm);
  h->comm = nullptr;
}

// Best-GT score keys for the MAX all-reduce (cmve_gt_thresholds' per-shard encoding: NaN = no GT in
// this shard, +inf = GTs here but every one scores NaN, else the best finite score).  Encoded, a finite
// score beats "all NaN" (-1e300), which beats "no GT" (-inf); RCCL's MAX never sees a NaN.
constexpr double NAN_GT_KEY = -1e300;

__global__ __launch_bounds__(256) void gt_key_kernel(double* __restrict__ s, int64_t n, int decode) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double v = s[i];
  if (!decode) {
    if (v != v) s[i] = -INFINITY;
    else if (v == INFINITY) s[i] = NAN_GT_KEY;
  } else {
    if (v == -INFINITY) s[i] = (double)NAN;
    else if (v == NAN_GT_KEY) s[i] = INFINITY;
  }
}

static int gt_keys(hipStream_t s, double* v, int64_t n, int decode) {
  if (n == 0) return CMVE_OK;
  hipLaunchKernelGGL(gt_key_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, v, n, decode);
  return check_launch("gt_key_kernel");
}

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_dist_unique_id(void* id) {
  CMVE_REQUIRE(id, "cmve_dist_unique_id: NULL output");
  const RcclApi* api = rccl_api();
  CMVE_REQUIRE(api, "cmve_dist_unique_id: RCCL (librccl.so) could not be opened");
  ncclUniqueId u;
  CMVE_RCCL(api, api->get_unique_id(&u), "cmve_dist_unique_id");
  memcpy(id, &u, sizeof(u));
  return CMVE_OK;
}

extern "C" int cmve_dist_init(cmve_handle_t h, int32_t nranks, int32_t rank, const void* id) {
  CMVE_REQUIRE(h && id, "cmve_dist_init: NULL handle / id");
  CMVE_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "cmve_dist_init: rank %d of %d", rank, nranks);
  CMVE_REQUIRE(!h->comm, "cmve_dist_init: the handle already holds a communicator");
  const RcclApi* api = rccl_api();
  CMVE_REQUIRE(api, "cmve_dist_init: RCCL (librccl.so) could not be opened");
  CMVE_HIP(hipSetDevice(h->device));
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t comm = nullptr;
  CMVE_RCCL(api, api->comm_init_rank(&comm, nranks, u, rank), "cmve_dist_init");
  h->comm = comm;
  h->nranks = nranks;
  h->rank = rank;
  return CMVE_OK;
}

extern "C" int cmve_dist_allgather_q(cmve_handle_t h, const float* local, int64_t n_local, int64_t d,
                                     float* gathered) {
  CMVE_REQUIRE(h && h->comm, "cmve_dist_allgather_q: handle has no communicator (cmve_dist_init)");
  CMVE_REQUIRE(n_local >= 0 && d > 0 && (n_local == 0 || (local && gathered)), "cmve_dist_allgather_q: bad argument");
  const RcclApi* api = rccl_api();
  CMVE_RCCL(api, api->all_gather(local, gathered, (size_t)(n_local * d), ncclFloat32, (ncclComm_t)h->comm, h->stream),
            "cmve_dist_allgather_q");
  return CMVE_OK;
}

extern "C" int cmve_dist_reduce_rank(cmve_handle_t h, double* best_gt, int32_t* counts, int64_t n) {
  CMVE_REQUIRE(h && h->comm, "cmve_dist_reduce_rank: handle has no communicator (cmve_dist_init)");
  CMVE_REQUIRE(n >= 0 && (n == 0 || best_gt || counts), "cmve_dist_reduce_rank: bad argument");
  const RcclApi* api = rccl_api();
  if (best_gt) {  // encode -> MAX -> decode, all on the handle's stream
    int st = gt_keys(h->stream, best_gt, n, 0);
    if (st) return st;
    CMVE_RCCL(api, api->all_reduce(best_gt, best_gt, (size_t)n, ncclFloat64, ncclMax, (ncclComm_t)h->comm, h->stream),
              "cmve_dist_reduce_rank (max)");
    st = gt_keys(h->stream, best_gt, n, 1);
    if (st) return st;
  }
  if (counts)
    CMVE_RCCL(api, api->all_reduce(counts, counts, (size_t)n, ncclInt32, ncclSum, (ncclComm_t)h->comm, h->stream),
              "cmve_dist_reduce_rank (sum)");
  return CMVE_OK;
}

extern "C" int cmve_dist_allgather_topk(cmve_handle_t h, const int64_t* ids, const double* scores, int64_t n_q,
                                        int32_t k, int64_t* gathered_ids, double* gathered_scores, int32_t k_out,
                                        int64_t* out_ids, double* out_scores) {
  CMVE_REQUIRE(h && h->comm, "cmve_dist_allgather_topk: handle has no communicator (cmve_dist_init)");
  CMVE_REQUIRE(n_q >= 0 && k >= 1 && k_out >= 1 && h->nranks <= 64, "cmve_dist_allgather_topk: bad argument");
  if (n_q == 0) return CMVE_OK;
  CMVE_REQUIRE(ids && scores && gathered_ids && gathered_scores && out_ids && out_scores,
               "cmve_dist_allgather_topk: NULL argument");
  const RcclApi* api = rccl_api();
  const size_t cnt = (size_t)(n_q * k);
  CMVE_RCCL(api, api->all_gather(ids, gathered_ids, cnt, ncclInt64, (ncclComm_t)h->comm, h->stream),
            "cmve_dist_allgather_topk (ids)");
  CMVE_RCCL(api, api->all_gather(scores, gathered_scores, cnt, ncclFloat64, (ncclComm_t)h->comm, h->stream),
            "cmve_dist_allgather_topk (scores)");
  // rank-major [nranks][n_q][k]: query q's run from rank r starts at r * n_q * k + q * k
  return merge_topk_launch(h->stream, gathered_ids, gathered_scores, n_q, h->nranks, k, k, (int64_t)n_q * k, k_out,
                           out_ids, out_scores);
}

// the plain collectives a host needs beside the three above (the two-direction exchange's SUM carries int64
// counts and R@K sums; the layout check and the v2t rank gather move int64 rows)
static bool nccl_type(int32_t dt, ncclDataType_t& t) {
  switch (dt) {
    case CMVE_F32: t = ncclFloat32; return true;
    case CMVE_F64: t = ncclFloat64; return true;
    case CMVE_I32: t = ncclInt32; return true;
    case CMVE_I64: t = ncclInt64; return true;
    default: return false;
  }
}

extern "C" int cmve_dist_allreduce(cmve_handle_t h, void* buf, int64_t count, int32_t dtype, int32_t op) {
  CMVE_REQUIRE(h && h->comm, "cmve_dist_allreduce: handle has no communicator (cmve_dist_init)");
  ncclDataType_t t;
  CMVE_REQUIRE(nccl_type(dtype, t), "cmve_dist_allreduce: unsupported dtype %d", dtype);
  CMVE_REQUIRE(op == CMVE_DIST_SUM || op == CMVE_DIST_MAX, "cmve_dist_allreduce: op must be SUM or MAX");
  CMVE_REQUIRE(count >= 0 && (count == 0 || buf), "cmve_dist_allreduce: bad argument");
  if (count == 0) return CMVE_OK;
  const RcclApi* api = rccl_api();
  CMVE_RCCL(api, api->all_reduce(buf, buf, (size_t)count, t, op == CMVE_DIST_SUM ? ncclSum : ncclMax,
                                 (ncclComm_t)h->comm, h->stream),
            "cmve_dist_allreduce");
  return CMVE_OK;
}

extern "C" int cmve_dist_allgather(cmve_handle_t h, const void* local, int64_t count, int32_t dtype, void* gathered) {
  CMVE_REQUIRE(h && h->comm, "cmve_dist_allgather: handle has no communicator (cmve_dist_init)");
  ncclDataType_t t;
  CMVE_REQUIRE(nccl_type(dtype, t), "cmve_dist_allgather: unsupported dtype %d", dtype);
  CMVE_REQUIRE(count >= 0 && (count == 0 || (local && gathered)), "cmve_dist_allgather: bad argument");
  if (count == 0) return CMVE_OK;
  const RcclApi* api = rccl_api();
  CMVE_RCCL(api, api->all_gather(local, gathered, (size_t)count, t, (ncclComm_t)h->comm, h->stream),
            "cmve_dist_allgather");
  return CMVE_OK;
}

extern "C" int cmve_dist_size(cmve_handle_t h, int32_t* nranks, int32_t* rank) {
  CMVE_REQUIRE(h && nranks && rank, "cmve_dist_size: NULL argument");
  CMVE_REQUIRE(h->comm, "cmve_dist_size: handle has no communicator (cmve_dist_init)");
  *nranks = h->nranks;
  *rank = h->rank;
  return CMVE_OK;
}

extern "C" int cmve_dist_destroy(cmve_handle_t h) {
  CMVE_REQUIRE(h, "cmve_dist_destroy: NULL handle");
  dist_release(h);
  return CMVE_OK;
}
