// K10: all-pairs non-cosine measures -- the non-GEMM similarity matrices of
//   LINAS-engine/evaluation.py:17-35,41-72   cal_error / cal_error_batch: scipy cdist 'euclidean',
//                                            'minkowski' p=1, their /D - 1 normalised forms, and
//                                            -jaccard (torch fp32)
//   LINAS-engine/loss.py:13-73               order / euclidean / L1 / L1_norm / L2 / L2_norm /
//                                            jaccard training similarities
// out[i, j] = alpha * f(a_i, b_j) + beta with
//   SQ_L2   f = sum_k (a_k - b_k)^2              L2   f = sqrt(SQ_L2)
//   L1      f = sum_k |a_k - b_k|                ORDER f = sqrt(sum_k max(0, b_k - a_k)^2)
//   JACCARD f = sum_k min(a_k, b_k) / sum_k max(a_k, b_k)
//   DOT     f = sum_k a_k b_k (k-ordered fp64 fma chain: the top-k's exact dense fallback)
// No MFMA form exists for these reductions (min/max/abs per element): a VALU kernel with 64x128
// output tiles per 256-thread block, 4x8 outputs per thread, K staged through LDS in 32-deep
// slabs (converted to fp64 once on the way in), fp64 accumulation -- the reference's scipy path
// is fp64 (encode_* buffers are fp64, evaluation.py:102); its torch paths are fp32 and agree to
// fp32 rounding.
#include "cmve_internal.h"

namespace cmve {

// Block tile 64 (A rows) x 128 (B rows), 256 threads as 16 x 16; thread (tx, ty) owns A rows
// {2ty + 32u + e} and B rows {2tx + 32v + e} (u < 2, v < 4, e < 2): 4 x 8 = 32 outputs from 2 + 4
// ds_read_b128 per k (16-B pairs, consecutive across the 16 lanes of a row group: conflict-free),
// against 8 ds_read_b64 per 16 outputs in a 4 x 4 layout -- the LDS port no longer matches the
// fp64 VALU rate.
constexpr int PW_TA = 64, PW_TB = 128, PW_K = 32, PW_PA = PW_TA + 2, PW_PB = PW_TB + 2;

template <int METRIC>
__device__ __forceinline__ void pw_acc(double a, double b, double& s0, double& s1) {
  if constexpr (METRIC == CMVE_PW_SQ_L2 || METRIC == CMVE_PW_L2) {
    const double t = a - b;
    s0 = fma(t, t, s0);
  } else if constexpr (METRIC == CMVE_PW_L1) {
    s0 += fabs(a - b);
  } else if constexpr (METRIC == CMVE_PW_ORDER) {
    const double t = fmax(b - a, 0.0);
    s0 = fma(t, t, s0);
  } else if constexpr (METRIC == CMVE_PW_DOT) {
    s0 = fma(a, b, s0);
  } else {  // JACCARD
    s0 += fmin(a, b);
    s1 += fmax(a, b);
  }
}

template <int METRIC>
__device__ __forceinline__ double pw_final(double s0, double s1) {
  if constexpr (METRIC == CMVE_PW_L2 || METRIC == CMVE_PW_ORDER) return sqrt(s0);
  else if constexpr (METRIC == CMVE_PW_JACCARD) return s0 / s1;
  else return s0;
}

template <typename TA, typename TB, typename TO, int METRIC>
__global__ __launch_bounds__(256) void pairwise_kernel(const TA* __restrict__ A, int64_t lda, int64_t na,
                                                       const TB* __restrict__ B, int64_t ldb, int64_t nb, int64_t d,
                                                       double alpha, double beta, TO* __restrict__ out,
                                                       int64_t ldo) {
  __shared__ __attribute__((aligned(16))) double sa[PW_K][PW_PA];  // [k][row], converted to fp64 once
  __shared__ __attribute__((aligned(16))) double sb[PW_K][PW_PB];
  constexpr bool JAC = METRIC == CMVE_PW_JACCARD;
  const int tid = threadIdx.x;
  const int tx = tid & 15, ty = tid >> 4;
  const int64_t i0 = (int64_t)blockIdx.y * PW_TA, j0 = (int64_t)blockIdx.x * PW_TB;
  double s0[4][8] = {}, s1[JAC ? 4 : 1][JAC ? 8 : 1] = {};
  for (int64_t k0 = 0; k0 < d; k0 += PW_K) {
    for (int e = tid; e < PW_TA * PW_K; e += 256) {  // coalesced along k
      const int r = e / PW_K, k = e % PW_K;
      const int64_t kk = k0 + k;
      sa[k][r] = (i0 + r < na && kk < d) ? (double)A[(i0 + r) * lda + kk] : 0.0;
    }
    for (int e = tid; e < PW_TB * PW_K; e += 256) {
      const int r = e / PW_K, k = e % PW_K;
      const int64_t kk = k0 + k;
      sb[k][r] = (j0 + r < nb && kk < d) ? (double)B[(j0 + r) * ldb + kk] : 0.0;
    }
    __syncthreads();
    const int kn = (int)min<int64_t>(PW_K, d - k0);  // zero padding would bias L1 / jaccard: stop at d
    for (int k = 0; k < kn; ++k) {
      double av[4], bv[8];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const double2 t = *(const double2*)&sa[k][2 * ty + 32 * u];
        av[2 * u] = t.x;
        av[2 * u + 1] = t.y;
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const double2 t = *(const double2*)&sb[k][2 * tx + 32 * v];
        bv[2 * v] = t.x;
        bv[2 * v + 1] = t.y;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 8; ++v) {
          double dummy = 0.0;
          pw_acc<METRIC>(av[u], bv[v], s0[u][v], JAC ? s1[JAC ? u : 0][JAC ? v : 0] : dummy);
        }
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = i0 + 2 * ty + 32 * (u >> 1) + (u & 1);
    if (i >= na) continue;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const int64_t j = j0 + 2 * tx + 32 * (v >> 1) + (v & 1);
      if (j < nb)
        out[i * ldo + j] =
            (TO)(alpha * pw_final<METRIC>(s0[u][v], JAC ? s1[JAC ? u : 0][JAC ? v : 0] : 0.0) + beta);
    }
  }
}

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_pairwise(cmve_handle_t h, const void* A, int32_t a_dtype, int64_t lda, int64_t na, const void* B,
                             int32_t b_dtype, int64_t ldb, int64_t nb, int64_t d, int32_t metric, double alpha,
                             double beta, void* out, int32_t out_dtype, int64_t ldo) {
  CMVE_REQUIRE(h && A && B && out, "cmve_pairwise: NULL argument");
  CMVE_REQUIRE(na >= 0 && nb >= 0 && d > 0 && lda >= d && ldb >= d && ldo >= nb, "cmve_pairwise: bad shape");
  CMVE_REQUIRE(metric >= CMVE_PW_SQ_L2 && metric <= CMVE_PW_DOT, "cmve_pairwise: unknown metric %d", metric);
  CMVE_REQUIRE((a_dtype == CMVE_F32 || a_dtype == CMVE_F64) && (b_dtype == CMVE_F32 || b_dtype == CMVE_F64) &&
                   (out_dtype == CMVE_F32 || out_dtype == CMVE_F64),
               "cmve_pairwise: dtypes must be CMVE_F32/CMVE_F64");
  if (na == 0 || nb == 0) return CMVE_OK;
  CMVE_REQUIRE((na + PW_TA - 1) / PW_TA < 65536, "cmve_pairwise: too many rows in A (%lld)", (long long)na);
  const dim3 grid((unsigned)((nb + PW_TB - 1) / PW_TB), (unsigned)((na + PW_TA - 1) / PW_TA));
#define PW_LAUNCH(TA, TB, TO, M)                                                                            \
  hipLaunchKernelGGL((pairwise_kernel<TA, TB, TO, M>), grid, dim3(256), 0, h->stream, (const TA*)A, lda, na, \
                     (const TB*)B, ldb, nb, d, alpha, beta, (TO*)out, ldo)
#define PW_METRIC(TA, TB, TO)                                          \
  switch (metric) {                                                    \
    case CMVE_PW_SQ_L2: PW_LAUNCH(TA, TB, TO, CMVE_PW_SQ_L2); break;   \
    case CMVE_PW_L2: PW_LAUNCH(TA, TB, TO, CMVE_PW_L2); break;         \
    case CMVE_PW_L1: PW_LAUNCH(TA, TB, TO, CMVE_PW_L1); break;         \
    case CMVE_PW_ORDER: PW_LAUNCH(TA, TB, TO, CMVE_PW_ORDER); break;   \
    case CMVE_PW_DOT: PW_LAUNCH(TA, TB, TO, CMVE_PW_DOT); break;       \
    default: PW_LAUNCH(TA, TB, TO, CMVE_PW_JACCARD); break;            \
  }
#define PW_OUT(TA, TB)              \
  if (out_dtype == CMVE_F64) {      \
    PW_METRIC(TA, TB, double)       \
  } else {                          \
    PW_METRIC(TA, TB, float)        \
  }
  if (a_dtype == CMVE_F64 && b_dtype == CMVE_F64) {
    PW_OUT(double, double)
  } else if (a_dtype == CMVE_F64) {
    PW_OUT(double, float)
  } else if (b_dtype == CMVE_F64) {
    PW_OUT(float, double)
  } else {
    PW_OUT(float, float)
  }
#undef PW_OUT
#undef PW_METRIC
#undef PW_LAUNCH
  return check_launch("pairwise");
}
