// K6 / K7: contrastive losses over a B x B score matrix S (rows = videos im / predictions,
// columns = captions s / targets), forward + backward, plus an exact-fp32 MFMA GEMM for the
// gradient products dL/dim = dS . s and dL/ds = dS^T . im (and the training heads' GEMMs, K11).
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
//   K15 element-pair losses of the distillation step (LINAS-engine/model.py:554-580,845-895):
//       MSE (x-y)^2 (nn.MSELoss), SmoothL1 beta 1 (nn.SmoothL1Loss: 0.5 d^2 if |d| < 1 else |d| - 0.5),
//       KLDiv (nn.KLDivLoss, log_target False: xlogy(y, y) - y x -- NaN for y < 0, as torch), each
//       optionally weighted per element (the 'diag' / 'adapt' similarity variants) and scaled
//       (sum / mean / * batchsize); backward d/dx and d/dy with torch's formulas.
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
    // d/dS_ii of -S_ii in every active row-i / column-i term.  max_violation: only the argmax term of
    // row i and of column i can be active (O(1)); sum style: triplet_diag_sum_kernel writes the diagonal.
    if (!max_violation) return;
    float cnt = 0.f;
    if (dir & 1) {
      const int k = rarg[i];
      if (k != i && margin + S[(int64_t)i * ld + k] - sij >= 0.f) cnt += 1.f;
    }
    if (dir & 2) {
      const int k = carg[i];
      if (k != i && margin + S[(int64_t)k * ld + i] - sij >= 0.f) cnt += 1.f;
    }
    v -= gr * cnt;
  }
  dS[(int64_t)i * ldd + j] = v;
}

// sum style: dS_ii = -g * (#active costs in row i + #active costs in column i), one wave per i
__global__ __launch_bounds__(256) void triplet_diag_sum_kernel(const float* __restrict__ S, int64_t ld, int B,
                                                               float margin, int dir, float wscale,
                                                               const float* __restrict__ g, float* __restrict__ dS,
                                                               int64_t ldd) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= B) return;
  const float sii = S[(int64_t)i * ld + i];
  int cnt = 0;
  for (int k = lane; k < B; k += 64) {
    if (k == i) continue;
    if ((dir & 1) && margin + S[(int64_t)i * ld + k] - sii >= 0.f) ++cnt;
    if ((dir & 2) && margin + S[(int64_t)k * ld + i] - sii >= 0.f) ++cnt;
  }
  cnt = wave_sum_i(cnt);
  if (lane == 0) dS[(int64_t)i * ldd + i] = -(g[0] * wscale) * (float)cnt;
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
// C = alpha * op(A) . op(B) + beta * C (+ bias[n]) (relu), on v_mfma_f32_16x16x4_f32: each
// K-slice is bit-for-bit a k-ordered fp32 fmaf chain (cdna_hip_programming.md, FP32-input MFMA).
// 64 x 64 block tile, 4 waves of 32 x 32 (2 x 2 MFMA tiles = 4 independent accumulators), K staged
// through LDS 32 at a time as [k][m] / [k][n] (+4 pad); global loads coalesced along whichever
// dimension is contiguous (float4 when every operand allows it).
// Split-K: small M x N grids (the B x B score GEMMs, B x 1024 projections) cannot fill 256 CUs with
// one serial K loop per tile, so blockIdx.z takes a K-slice and writes raw partials to scratch;
// gemm_splitk_reduce_kernel sums the slices in fixed z order (deterministic) and applies the epilogue.
typedef float gf32x4 __attribute__((ext_vector_type(4)));
constexpr int GT = 64, GK = 32, GP = GT + 4;

template <bool VEC>
__device__ __forceinline__ void gemm_stage(const float* __restrict__ X, int64_t ldx, bool kmajor, int r0, int R,
                                           int k0, int K, float (*S)[GP]) {
  // stage op(X)[r0 .. r0+64)[k0 .. k0+32) into S[k][r]; kmajor: X[k][r] (r contiguous), else X[r][k]
  const int tid = threadIdx.x;
  if constexpr (VEC) {
#pragma unroll
    for (int e = 0; e < GT * GK / 1024; ++e) {
      const int idx = e * 256 + tid;  // float4 index
      if (kmajor) {
        const int kk = idx / (GT / 4), rr = (idx % (GT / 4)) * 4;
        const int gk = k0 + kk, gr = r0 + rr;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gk < K && gr < R) v = *reinterpret_cast<const float4*>(X + (int64_t)gk * ldx + gr);
        S[kk][rr] = v.x; S[kk][rr + 1] = v.y; S[kk][rr + 2] = v.z; S[kk][rr + 3] = v.w;
      } else {
        const int rr = idx / (GK / 4), kk = (idx % (GK / 4)) * 4;
        const int gk = k0 + kk, gr = r0 + rr;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gk < K && gr < R) v = *reinterpret_cast<const float4*>(X + (int64_t)gr * ldx + gk);
        S[kk][rr] = v.x; S[kk + 1][rr] = v.y; S[kk + 2][rr] = v.z; S[kk + 3][rr] = v.w;
      }
    }
  } else {
#pragma unroll
    for (int e = 0; e < GT * GK / 256; ++e) {
      const int idx = e * 256 + tid;
      int rr, kk;
      if (kmajor) { kk = idx / GT; rr = idx % GT; } else { rr = idx / GK; kk = idx % GK; }
      const int gr = r0 + rr, gk = k0 + kk;
      float v = 0.f;
      if (gr < R && gk < K) v = kmajor ? X[(int64_t)gk * ldx + gr] : X[(int64_t)gr * ldx + gk];
      S[kk][rr] = v;
    }
  }
}

template <bool VEC>
__global__ __launch_bounds__(256) void gemm_f32_kernel(int transA, int transB, int M, int N, int K, int kslice,
                                                       float alpha, const float* __restrict__ A, int64_t lda,
                                                       const float* __restrict__ Bm, int64_t ldb, float beta,
                                                       float* __restrict__ C, int64_t ldc,
                                                       const float* __restrict__ bias, int relu,
                                                       float* __restrict__ part) {
  __shared__ float As[GK][GP];
  __shared__ float Bs[GK][GP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int kb = blockIdx.z * kslice, ke = min(K, kb + kslice);
  gf32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = gf32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = kb; k0 < ke; k0 += GK) {
    gemm_stage<VEC>(A, lda, transA != 0, m0, M, k0, ke, As);    // op(A)[m][k]
    gemm_stage<VEC>(Bm, ldb, transB == 0, n0, N, k0, ke, Bs);   // op(B)[k][n]: B[k][n] is n-contiguous
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < GK; ks += 4) {
      const int kr = ks + (lane >> 4);
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = As[kr][wm + i * 16 + (lane & 15)];
        b[i] = Bs[kr][wn + i * 16 + (lane & 15)];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // C/D map of 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int gn = n0 + wn + j * 16 + (lane & 15);
      if (gn >= N) continue;
      const float bn = (bias && !part) ? bias[gn] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
        if (gm >= M) continue;
        if (part) {
          part[((int64_t)blockIdx.z * M + gm) * N + gn] = acc[i][j][r];
        } else {
          float* c = C + (int64_t)gm * ldc + gn;
          float v = alpha * acc[i][j][r] + (beta != 0.f ? beta * *c : 0.f) + bn;
          if (relu) v = v > 0.f ? v : 0.f;
          *c = v;
        }
      }
    }
}

__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(const float* __restrict__ part, int splits, int M,
                                                                 int N, float alpha, float beta,
                                                                 float* __restrict__ C, int64_t ldc,
                                                                 const float* __restrict__ bias, int relu) {
  const int64_t total = (int64_t)M * N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    float s = part[i];
    for (int z = 1; z < splits; ++z) s += part[(int64_t)z * total + i];
    const int gm = (int)(i / N), gn = (int)(i % N);
    float* c = C + (int64_t)gm * ldc + gn;
    float v = alpha * s + (beta != 0.f ? beta * *c : 0.f) + (bias ? bias[gn] : 0.f);
    if (relu) v = v > 0.f ? v : 0.f;
    *c = v;
  }
}

// ---------------- K15: element-pair losses ----------------
__device__ __forceinline__ float pair_f(int kind, float x, float y) {
  if (kind == 0) {
    const float d = x - y;
    return d * d;
  }
  if (kind == 1) {
    const float d = x - y, a = fabsf(d);
    return a < 1.f ? 0.5f * d * d : a - 0.5f;
  }
  // xlogy(y, y) - y * x: 0 * log 0 = 0, log of a negative target is NaN
  const float xl = (y == 0.f) ? 0.f : y * logf(y);
  return xl - y * x;
}

__global__ __launch_bounds__(1024) void pair_loss_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                         const float* __restrict__ w, int64_t n, int kind, float scale,
                                                         float* __restrict__ loss) {
  __shared__ double red[16];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 1024) {
    float f = pair_f(kind, x[i], y[i]);
    if (w) f *= w[i];
    s += (double)f;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < 16; ++k) t += red[k];
    loss[0] = (float)(t * (double)scale);
  }
}

__global__ __launch_bounds__(256) void pair_grad_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                        const float* __restrict__ w, int64_t n, int kind, float scale,
                                                        const float* __restrict__ g, float* __restrict__ dx,
                                                        float* __restrict__ dy) {
  const float gs = g[0] * scale;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float xv = x[i], yv = y[i];
    float gx, gy;
    if (kind == 0) {
      gx = 2.f * (xv - yv);
      gy = -gx;
    } else if (kind == 1) {
      const float d = xv - yv;
      gx = d < -1.f ? -1.f : (d > 1.f ? 1.f : d);
      gy = -gx;
    } else {
      gx = -yv;
      gy = yv > 0.f ? logf(yv) + 1.f - xv : NAN;
    }
    const float c = w ? gs * w[i] : gs;
    if (dx) dx[i] = c * gx;
    if (dy) dy[i] = c * gy;
  }
}

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_pair_loss_fwd(cmve_handle_t h, const float* x, const float* y, const float* w, int64_t n,
                                  int32_t kind, float scale, float* loss) {
  CMVE_REQUIRE(h && loss && (n == 0 || (x && y)), "cmve_pair_loss_fwd: NULL argument");
  CMVE_REQUIRE(n >= 0 && kind >= 0 && kind <= 2, "cmve_pair_loss_fwd: bad size / kind %d", kind);
  hipLaunchKernelGGL(pair_loss_kernel, dim3(1), dim3(1024), 0, h->stream, x, y, w, n, kind, scale, loss);
  return check_launch("pair_loss_fwd");
}

extern "C" int cmve_pair_loss_bwd(cmve_handle_t h, const float* x, const float* y, const float* w, int64_t n,
                                  int32_t kind, float scale, const float* g, float* dx, float* dy) {
  CMVE_REQUIRE(h && g && (n == 0 || (x && y)), "cmve_pair_loss_bwd: NULL argument");
  CMVE_REQUIRE(n >= 0 && kind >= 0 && kind <= 2, "cmve_pair_loss_bwd: bad size / kind %d", kind);
  if (n == 0 || (!dx && !dy)) return CMVE_OK;
  const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(pair_grad_kernel, dim3(blocks), dim3(256), 0, h->stream, x, y, w, n, kind, scale, g, dx, dy);
  return check_launch("pair_loss_bwd");
}

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
  if (!max_violation)
    hipLaunchKernelGGL(triplet_diag_sum_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, h->stream, S, ld, B, margin,
                       dir, wscale, g, dS, ldd);
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

static int gemm_f32_launch(cmve_handle_t h, int32_t transA, int32_t transB, int64_t M, int64_t N, int64_t K,
                           float alpha, const float* A, int64_t lda, const float* B, int64_t ldb, float beta, float* C,
                           int64_t ldc, const float* bias, int32_t relu, const char* who) {
  CMVE_REQUIRE(h && A && B && C, "%s: NULL argument", who);
  CMVE_REQUIRE(M >= 0 && N >= 0 && K >= 0 && M < (1 << 30) && N < (1 << 30) && K < (1 << 30), "%s: bad shape", who);
  CMVE_REQUIRE(ldc >= N && lda >= (transA ? M : K) && ldb >= (transB ? K : N), "%s: leading dimension too small", who);
  if (M == 0 || N == 0) return CMVE_OK;
  CMVE_REQUIRE((M + GT - 1) / GT < 65536, "%s: M too large for the grid", who);
  const int64_t nbm = (M + GT - 1) / GT, nbn = (N + GT - 1) / GT, blocks = nbm * nbn;
  // split K until the grid reaches ~2 blocks per CU, keeping >= 2 K-tiles per slice
  int64_t splits = 1;
  while (blocks * splits * 2 <= 512 && K / (splits * 2) >= 2 * GK) splits *= 2;
  const int64_t kslice = ((K + splits * GK - 1) / (splits * GK)) * GK;
  splits = std::max<int64_t>(1, (K + kslice - 1) / kslice);
  float* part = nullptr;
  if (splits > 1) {
    const int rc = ensure_scratch(h, (size_t)splits * M * N * sizeof(float));
    if (rc != CMVE_OK) return rc;
    part = (float*)h->scratch;
  }
  // float4 staging needs 16-B aligned rows and 4-multiples along every contiguous extent
  auto al = [](const void* p, int64_t ld) { return ((uintptr_t)p % 16 == 0) && (ld % 4 == 0); };
  const bool vec = al(A, lda) && al(B, ldb) && (transA ? M % 4 == 0 : K % 4 == 0) && (transB ? K % 4 == 0 : N % 4 == 0);
  dim3 grid((unsigned)nbn, (unsigned)nbm, (unsigned)splits);
  if (vec)
    hipLaunchKernelGGL(gemm_f32_kernel<true>, grid, dim3(256), 0, h->stream, transA, transB, (int)M, (int)N, (int)K,
                       (int)kslice, alpha, A, lda, B, ldb, beta, C, ldc, bias, relu, part);
  else
    hipLaunchKernelGGL(gemm_f32_kernel<false>, grid, dim3(256), 0, h->stream, transA, transB, (int)M, (int)N, (int)K,
                       (int)kslice, alpha, A, lda, B, ldb, beta, C, ldc, bias, relu, part);
  if (splits > 1)
    hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3((unsigned)std::min<int64_t>((M * N + 255) / 256, 2048)),
                       dim3(256), 0, h->stream, part, (int)splits, (int)M, (int)N, alpha, beta, C, ldc, bias, relu);
  return check_launch(who);
}

extern "C" int cmve_gemm_f32(cmve_handle_t h, int32_t transA, int32_t transB, int64_t M, int64_t N, int64_t K, float alpha,
                             const float* A, int64_t lda, const float* B, int64_t ldb, float beta, float* C,
                             int64_t ldc) {
  return gemm_f32_launch(h, transA, transB, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, nullptr, 0, "cmve_gemm_f32");
}

extern "C" int cmve_gemm_f32_ex(cmve_handle_t h, int32_t transA, int32_t transB, int64_t M, int64_t N, int64_t K,
                                float alpha, const float* A, int64_t lda, const float* B, int64_t ldb, float beta,
                                float* C, int64_t ldc, const float* bias, int32_t relu) {
  return gemm_f32_launch(h, transA, transB, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, bias, relu,
                         "cmve_gemm_f32_ex");
}
