// K6 / K7: contrastive losses over a B x B score matrix S (rows = videos im / predictions,
// columns = captions s / targets), forward + backward, plus a tiled fp32 GEMM for the
// gradient products dL/dim = dS . s and dL/ds = dS^T . im.
//
//   K6  TripletLoss  LINAS-engine/loss.py:83-153
//       cost_s [i,j] = [m + S_ij - S_ii]_+ (j != i), reduced over j (dim 1)   direction v2t
//       cost_im[i,j] = [m + S_ij - S_jj]_+ (i != j), reduced over i (dim 0)   direction t2v
//       max_violation: max (first index on ties, as torch.max); else the sum of all costs;
//       cost_style sum | mean.  Backward follows autograd: clamp passes where m + S_ij - S_dd >= 0,
//       masked_fill_ zeroes the diagonal, max routes to its argmax.
//   K7  InfoNCE      MultiFusion/src/combiner_train.py:318,367-372 (CE(100 * P.T^T, arange): row half)
//       and its transpose (MCT/mmaction/models/backbones/clip.py:383-386): the col half.
//       loss_row = mean_i (lse_j(t S_ij) - t S_ii), loss_col = mean_j (lse_i(t S_ij) - t S_jj).
// Reductions are deterministic (fixed order, single block for the final sum).
#include "cmve_internal.h"

namespace cmve {

// ---------------- TripletLoss ----------------
// one wave per row (dir bit 1) / per column (dir bit 2)
__global__ __launch_bounds__(256) void triplet_reduce_kernel(const float* __restrict__ S, int64_t ld, int B,
                                                             float margin, int max_violation, int cols,
                                                             float* __restrict__ val, int* __restrict__ arg) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  const float d = S[(int64_t)r * ld + r];
  float best = -INFINITY;
  int bi = 0x7fffffff;
  float sum = 0.f;
  for (int k = lane; k < B; k += 64) {
    const float x = cols ? S[(int64_t)k * ld + r] : S[(int64_t)r * ld + k];
    float c = margin + x - d;  // (margin + scores) - d, as loss.py:130/135 evaluates it
    c = c > 0.f ? c : 0.f;
    if (k == r) c = 0.f;  // masked_fill_(I, 0)
    if (max_violation) {
      if (c > best) { best = c; bi = k; }
    } else {
      sum += c;
    }
  }
  if (max_violation) {
    for (int o = 32; o >= 1; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (lane == 0) { val[r] = best; arg[r] = bi; }
  } else {
    // fixed-order pairwise reduction
    for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (lane == 0) { val[r] = sum; arg[r] = -1; }
  }
}

// loss = reduce(val_row) + reduce(val_col), sum or mean; single block, fixed order
__global__ __launch_bounds__(256) void sum2_kernel(const float* __restrict__ a, int na, float sa,
                                                   const float* __restrict__ b, int nb, float sb,
                                                   float* __restrict__ out) {
  __shared__ double part[256];
  double acc_a = 0.0, acc_b = 0.0;
  for (int i = threadIdx.x; i < na; i += 256) acc_a += (double)a[i];
  for (int i = threadIdx.x; i < nb; i += 256) acc_b += (double)b[i];
  part[threadIdx.x] = acc_a * sa + acc_b * sb;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)part[0];
}

// dS for the triplet loss (dense, B x B), upstream gradient g[0]
__global__ __launch_bounds__(256) void triplet_grad_kernel(const float* __restrict__ S, int64_t ld, int B,
                                                           float margin, int max_violation, int dir, float wscale,
                                                           const float* __restrict__ g,
                                                           const int* __restrict__ rarg, const int* __restrict__ carg,
                                                           float* __restrict__ dS, int64_t ldd) {
  // one thread per element (i, j); diagonal gets the negated sums of its row/column terms
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)B * B) return;
  const int i = (int)(idx / B), j = (int)(idx % B);
  const float gr = g[0] * wscale;
  float v = 0.f;
  const float sij = S[(int64_t)i * ld + j];
  if (i != j) {
    if (dir & 1) {  // cost_s row i: m + S_ij - S_ii
      const bool act = max_violation ? (rarg[i] == j) : true;
      if (act && margin + sij - S[(int64_t)i * ld + i] >= 0.f) v += gr;
    }
    if (dir & 2) {  // cost_im column j: m + S_ij - S_jj
      const bool act = max_violation ? (carg[j] == i) : true;
      if (act && margin + sij - S[(int64_t)j * ld + j] >= 0.f) v += gr;
    }
  } else {
    // d/dS_ii of -S_ii in every active row-i term and every active column-i term
    float cnt = 0.f;
    for (int k = 0; k < B; ++k) {
      if (k == i) continue;
      if (dir & 1) {
        const bool act = max_violation ? (rarg[i] == k) : true;
        if (act && margin + S[(int64_t)i * ld + k] - sij >= 0.f) cnt += 1.f;
      }
      if (dir & 2) {
        const bool act = max_violation ? (carg[i] == k) : true;
        if (act && margin + S[(int64_t)k * ld + i] - sij >= 0.f) cnt += 1.f;
      }
    }
    v -= gr * cnt;
  }
  dS[(int64_t)i * ldd + j] = v;
}

// ---------------- InfoNCE ----------------
__global__ __launch_bounds__(256) void lse_kernel(const float* __restrict__ S, int64_t ld, int B, float t, int cols,
                                                  double* __restrict__ lse, float* __restrict__ loss) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  float m = -INFINITY;
  for (int k = lane; k < B; k += 64) {
    const float x = t * (cols ? S[(int64_t)k * ld + r] : S[(int64_t)r * ld + k]);
    m = fmaxf(m, x);
  }
  m = wave_max(m);
  double acc = 0.0;
  for (int k = lane; k < B; k += 64) {
    const float x = t * (cols ? S[(int64_t)k * ld + r] : S[(int64_t)r * ld + k]);
    acc += exp((double)x - (double)m);
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    const double l = (double)m + log(acc);
    lse[r] = l;
    loss[r] = (float)(l - (double)(t * S[(int64_t)r * ld + r]));
  }
}

// dS_ij = t * ( g_row/B * (softmax_row_ij - d_ij) + g_col/B * (softmax_col_ij - d_ij) )
__global__ __launch_bounds__(256) void infonce_grad_kernel(const float* __restrict__ S, int64_t ld, int B, float t,
                                                           int dir, const float* __restrict__ g,
                                                           const double* __restrict__ rlse,
                                                           const double* __restrict__ clse, float* __restrict__ dS,
                                                           int64_t ldd) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)B * B) return;
  const int i = (int)(idx / B), j = (int)(idx % B);
  const double x = (double)(t * S[(int64_t)i * ld + j]);
  const double delta = i == j ? 1.0 : 0.0;
  // dir 3 ('both') = (row + col) / 2
  const double w = dir == 3 ? 0.5 : 1.0;
  double v = 0.0;
  if (dir & 1) v += w * (exp(x - rlse[i]) - delta);
  if (dir & 2) v += w * (exp(x - clse[j]) - delta);
  dS[(int64_t)i * ldd + j] = (float)((double)g[0] * (double)t * v / (double)B);
}

__global__ __launch_bounds__(256) void infonce_combine_kernel(const float* __restrict__ rl, const float* __restrict__ cl,
                                                              int B, int dir, float* __restrict__ out) {
  __shared__ double pr[256], pc[256];
  double a = 0.0, b = 0.0;
  for (int i = threadIdx.x; i < B; i += 256) {
    if (dir & 1) a += (double)rl[i];
    if (dir & 2) b += (double)cl[i];
  }
  pr[threadIdx.x] = a;
  pc[threadIdx.x] = b;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      pr[threadIdx.x] += pr[threadIdx.x + s];
      pc[threadIdx.x] += pc[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double r = pr[0] / B, c = pc[0] / B;
    out[0] = (float)r;
    out[1] = (float)c;
    out[2] = (float)(dir == 3 ? 0.5 * (r + c) : (dir == 1 ? r : c));
  }
}

// ---------------- fp32 GEMM (gradient products) ----------------
// C[M,N] = alpha * op(A)[M,K] . B[K,N] + beta * C ; op(A) = A (transA=0, A[M,K]) or A^T (A[K,M]).
// 64x64 tiles, 256 threads x (4x4) outputs, K step 16 through LDS, fp32 FMA chain.
__global__ __launch_bounds__(256) void gemm_f32_kernel(int transA, int transB, int M, int N, int K, float alpha,
                                                       const float* __restrict__ A, int64_t lda,
                                                       const float* __restrict__ Bm, int64_t ldb, float beta,
                                                       float* __restrict__ C, int64_t ldc) {
  __shared__ float As[16][64 + 1];
  __shared__ float Bs[16][64 + 1];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += 16) {
    for (int e = threadIdx.x; e < 16 * 64; e += 256) {
      const int kk = e / 64, mm = e % 64;
      const int gm = m0 + mm, gk = k0 + kk;
      float av = 0.f;
      if (gm < M && gk < K) av = transA ? A[(int64_t)gk * lda + gm] : A[(int64_t)gm * lda + gk];
      As[kk][mm] = av;
      const int gn = n0 + mm;
      Bs[kk][mm] = (gn < N && gk < K) ? (transB ? Bm[(int64_t)gn * ldb + gk] : Bm[(int64_t)gk * ldb + gn]) : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = As[kk][ty * 4 + u];
        b[u] = Bs[kk][tx * 4 + u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = fmaf(a[u], b[v], acc[u][v]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int gm = m0 + ty * 4 + u, gn = n0 + tx * 4 + v;
      if (gm < M && gn < N) {
        float* c = C + (int64_t)gm * ldc + gn;
        *c = alpha * acc[u][v] + (beta != 0.f ? beta * *c : 0.f);
      }
    }
}

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_triplet_fwd(cmve_handle_t h, const float* S, int64_t ld, int32_t B, float margin,
                                int32_t max_violation, int32_t dir, int32_t mean_style, float* loss,
                                float* row_val, int32_t* row_arg, float* col_val, int32_t* col_arg) {
  CMVE_REQUIRE(h && S && loss && row_val && row_arg && col_val && col_arg, "cmve_triplet_fwd: NULL argument");
  CMVE_REQUIRE(B > 0 && ld >= B && (dir & ~3) == 0 && dir != 0, "cmve_triplet_fwd: bad shape / direction");
  dim3 grid((unsigned)((B + 3) / 4));
  if (dir & 1)
    hipLaunchKernelGGL(triplet_reduce_kernel, grid, dim3(256), 0, h->stream, S, ld, B, margin, max_violation, 0,
                       row_val, row_arg);
  if (dir & 2)
    hipLaunchKernelGGL(triplet_reduce_kernel, grid, dim3(256), 0, h->stream, S, ld, B, margin, max_violation, 1,
                       col_val, col_arg);
  // max_violation: vectors of B maxima; otherwise per-row sums (the mean over all B*B entries)
  const float scale = mean_style ? (max_violation ? 1.f / B : 1.f / ((float)B * (float)B)) : 1.f;
  hipLaunchKernelGGL(sum2_kernel, dim3(1), dim3(256), 0, h->stream, row_val, (dir & 1) ? B : 0, scale, col_val,
                     (dir & 2) ? B : 0, scale, loss);
  return check_launch("triplet_fwd");
}

extern "C" int cmve_triplet_bwd(cmve_handle_t h, const float* S, int64_t ld, int32_t B, float margin,
                                int32_t max_violation, int32_t dir, int32_t mean_style, const float* g,
                                const int32_t* row_arg, const int32_t* col_arg, float* dS, int64_t ldd) {
  CMVE_REQUIRE(h && S && g && dS, "cmve_triplet_bwd: NULL argument");
  CMVE_REQUIRE(B > 0 && ld >= B && ldd >= B, "cmve_triplet_bwd: bad shape");
  CMVE_REQUIRE(!max_violation || ((!(dir & 1) || row_arg) && (!(dir & 2) || col_arg)),
               "cmve_triplet_bwd: argmax arrays missing");
  // cost_style 'mean': the mean over B maxima (max_violation) or over all B*B costs
  const float wscale = mean_style ? (max_violation ? 1.f / (float)B : 1.f / ((float)B * (float)B)) : 1.f;
  const int64_t n = (int64_t)B * B;
  hipLaunchKernelGGL(triplet_grad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream, S, ld, B,
                     margin, max_violation, dir, wscale, g, row_arg, col_arg, dS, ldd);
  return check_launch("triplet_bwd");
}

extern "C" int cmve_infonce_fwd(cmve_handle_t h, const float* S, int64_t ld, int32_t B, float scale, int32_t dir,
                                float* loss3, double* row_lse, double* col_lse, float* row_loss, float* col_loss) {
  CMVE_REQUIRE(h && S && loss3 && row_lse && col_lse && row_loss && col_loss, "cmve_infonce_fwd: NULL argument");
  CMVE_REQUIRE(B > 0 && ld >= B && (dir & ~3) == 0 && dir != 0, "cmve_infonce_fwd: bad shape / direction");
  dim3 grid((unsigned)((B + 3) / 4));
  if (dir & 1) hipLaunchKernelGGL(lse_kernel, grid, dim3(256), 0, h->stream, S, ld, B, scale, 0, row_lse, row_loss);
  if (dir & 2) hipLaunchKernelGGL(lse_kernel, grid, dim3(256), 0, h->stream, S, ld, B, scale, 1, col_lse, col_loss);
  hipLaunchKernelGGL(infonce_combine_kernel, dim3(1), dim3(256), 0, h->stream, row_loss, col_loss, B, dir, loss3);
  return check_launch("infonce_fwd");
}

extern "C" int cmve_infonce_bwd(cmve_handle_t h, const float* S, int64_t ld, int32_t B, float scale, int32_t dir,
                                const float* g, const double* row_lse, const double* col_lse, float* dS,
                                int64_t ldd) {
  CMVE_REQUIRE(h && S && g && dS && (!(dir & 1) || row_lse) && (!(dir & 2) || col_lse),
               "cmve_infonce_bwd: NULL argument");
  CMVE_REQUIRE(B > 0 && ld >= B && ldd >= B && (dir & ~3) == 0 && dir != 0, "cmve_infonce_bwd: bad shape");
  const int64_t n = (int64_t)B * B;
  hipLaunchKernelGGL(infonce_grad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream, S, ld, B,
                     scale, dir, g, row_lse, col_lse, dS, ldd);
  return check_launch("infonce_bwd");
}

extern "C" int cmve_gemm_f32(cmve_handle_t h, int32_t transA, int32_t transB, int64_t M, int64_t N, int64_t K, float alpha,
                             const float* A, int64_t lda, const float* B, int64_t ldb, float beta, float* C,
                             int64_t ldc) {
  CMVE_REQUIRE(h && A && B && C, "cmve_gemm_f32: NULL argument");
  CMVE_REQUIRE(M >= 0 && N >= 0 && K >= 0 && M < (1 << 30) && N < (1 << 30) && K < (1 << 30),
               "cmve_gemm_f32: bad shape");
  if (M == 0 || N == 0) return CMVE_OK;
  dim3 grid((unsigned)((N + 63) / 64), (unsigned)((M + 63) / 64));
  hipLaunchKernelGGL(gemm_f32_kernel, grid, dim3(256), 0, h->stream, transA, transB, (int)M, (int)N, (int)K, alpha, A, lda, B,
                     ldb, beta, C, ldc);
  return check_launch("gemm_f32");
}
