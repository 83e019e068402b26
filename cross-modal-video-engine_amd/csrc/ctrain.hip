// K16: the non-GEMM pieces of the MultiFusion Combiner's TRAINING step (MultiFusion/src/combiner_train.py:
// 341-381: combiner.train(); logits = combiner(ref, text, target); CE(logits, arange); backward; Adam),
// forward and backward.  The Linear / 1x1-conv / in-projection GEMMs run on cmve_gemm_f32(_ex) (K11's
// exact-fp32 MFMA GEMM), the CE on K7, dropout on K11; what is left is here:
//
//   cmve_act_fwd / _bwd        ReLU, Sigmoid, QuickGELU x*sigmoid(1.702x)        (combiner.py:8-9,104-105,151-176)
//   cmve_layernorm_train_fwd   LayerNorm keeping the row mean / rstd; _bwd: dx, dgamma, dbeta
//                              (ResidualAttentionBlock ln_1 / ln_2, combiner.py:11-17,38-43)
//   cmve_mha_1q_bwd            the one-query-per-batch-element attention of the block (q [B, H*dh],
//                              keys / values at rows t*B + b of kv: the raw p_s_m.reshape(l*f, b, d) of
//                              combiner.py:164-165), gradients of q, K and V; softmax recomputed
//   cmve_combine_train_fwd/_bwd output = ((y + ds*text) + (1-ds)*ref) + based  (combiner.py:178-179,
//                              before F.normalize), gradients of text, ref and ds
//   cmve_pool_mean_bwd         dx[b, t, :] = dy[b, :] / T  (time_process, combiner.py:140-143)
// fp64 accumulation for every reduction; one wave per row for the row-wise ones (deterministic).
#include "cmve_internal.h"

namespace cmve {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__global__ __launch_bounds__(256) void act_fwd_kernel(const float* __restrict__ x, int64_t n, int kind,
                                                      float* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = x[i];
    float r;
    if (kind == 0) r = v > 0.f ? v : 0.f;
    else if (kind == 1) r = sigm(v);
    else r = v * sigm(1.702f * v);
    y[i] = r;
  }
}

__global__ __launch_bounds__(256) void act_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                      int64_t n, int kind, float* __restrict__ dx) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = x[i], g = dy[i];
    float r;
    if (kind == 0) {
      r = v > 0.f ? g : 0.f;  // torch's threshold_backward: 0 at v == 0
    } else if (kind == 1) {
      const float s = sigm(v);
      r = g * (1.f - s) * s;  // sigmoid_backward: grad * (1 - y) * y
    } else {
      const float s = sigm(1.702f * v);  // d/dv [v s(1.702 v)] = s + v * 1.702 * s (1 - s)
      r = g * s + g * v * (1.702f * s * (1.f - s));
    }
    dx[i] = r;
  }
}

// one wave per row; mean / rstd in fp64, stored as fp32 for the backward
__global__ __launch_bounds__(256) void ln_train_fwd_kernel(const float* __restrict__ x, int64_t ldx, int64_t n,
                                                           int64_t d, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, double eps,
                                                           float* __restrict__ y, int64_t ldy,
                                                           float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const float* xr = x + row * ldx;
  double s = 0.0;
  for (int64_t k = lane; k < d; k += 64) s += (double)xr[k];
  const double mean = wave_sum(s) / (double)d;
  double q = 0.0;
  for (int64_t k = lane; k < d; k += 64) {
    const double c = (double)xr[k] - mean;
    q = fma(c, c, q);
  }
  const double rstd = 1.0 / sqrt(wave_sum(q) / (double)d + eps);
  float* yr = y + row * ldy;
  for (int64_t k = lane; k < d; k += 64) {
    const double c = ((double)xr[k] - mean) * rstd;
    yr[k] = (float)(c * (double)(gamma ? gamma[k] : 1.f) + (double)(beta ? beta[k] : 0.f));
  }
  if (lane == 0) {
    mean_out[row] = (float)mean;
    rstd_out[row] = (float)rstd;
  }
}

// dx = rstd * (g dy - mean(g dy) - xhat * mean(g dy xhat)), one wave per row
__global__ __launch_bounds__(256) void ln_bwd_dx_kernel(const float* __restrict__ x, int64_t ldx,
                                                        const float* __restrict__ dy, int64_t lddy, int64_t n,
                                                        int64_t d, const float* __restrict__ gamma,
                                                        const float* __restrict__ mean, const float* __restrict__ rstd,
                                                        float* __restrict__ dx, int64_t lddx) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const float* xr = x + row * ldx;
  const float* gr = dy + row * lddy;
  const double mu = mean[row], rs = rstd[row];
  double s1 = 0.0, s2 = 0.0;
  for (int64_t k = lane; k < d; k += 64) {
    const double gd = (double)gr[k] * (double)(gamma ? gamma[k] : 1.f);
    const double xh = ((double)xr[k] - mu) * rs;
    s1 += gd;
    s2 = fma(gd, xh, s2);
  }
  s1 = wave_sum(s1) / (double)d;
  s2 = wave_sum(s2) / (double)d;
  float* dr = dx + row * lddx;
  for (int64_t k = lane; k < d; k += 64) {
    const double gd = (double)gr[k] * (double)(gamma ? gamma[k] : 1.f);
    const double xh = ((double)xr[k] - mu) * rs;
    dr[k] = (float)(rs * (gd - s1 - xh * s2));
  }
}

// dgamma[k] = sum_rows dy * xhat, dbeta[k] = sum_rows dy: one thread per column, rows in order
__global__ __launch_bounds__(256) void ln_bwd_param_kernel(const float* __restrict__ x, int64_t ldx,
                                                           const float* __restrict__ dy, int64_t lddy, int64_t n,
                                                           int64_t d, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, float* __restrict__ dgamma,
                                                           float* __restrict__ dbeta) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= d) return;
  double sg = 0.0, sb = 0.0;
  for (int64_t r = 0; r < n; ++r) {
    const double g = (double)dy[r * lddy + k];
    const double xh = ((double)x[r * ldx + k] - (double)mean[r]) * (double)rstd[r];
    sg = fma(g, xh, sg);
    sb += g;
  }
  if (dgamma) dgamma[k] = (float)sg;
  if (dbeta) dbeta[k] = (float)sb;
}

// block per (b, h): recompute the T scores and the softmax (mha_1q_kernel's arithmetic), then
//   dv_t = p_t dout,  dp_t = dout . v_t,  ds_t = p_t (dp_t - sum_u p_u dp_u),
//   dk_t = ds_t * scaling * q,  dq = scaling * sum_t ds_t k_t
__global__ __launch_bounds__(256) void mha_1q_bwd_kernel(const float* __restrict__ q, int64_t ldq,
                                                         const float* __restrict__ kv, int64_t ldkv, int64_t v_off,
                                                         int B, int T, int H, int dh, const float* __restrict__ dout,
                                                         int64_t lddo, float* __restrict__ dq, int64_t lddq,
                                                         float* __restrict__ dkv, int64_t lddkv) {
  extern __shared__ float sh[];  // p[T] + dp[T] + qs[dh] + go[dh] + partial dq [4][dh]
  float* p = sh;
  float* dp = p + T;
  float* qs = dp + T;
  float* go = qs + dh;
  float* pq = go + dh;
  __shared__ double red;
  const int b = blockIdx.x, h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float scaling = 1.0f / sqrtf((float)dh);
  for (int e = tid; e < dh; e += 256) {
    qs[e] = q[(int64_t)b * ldq + h * dh + e] * scaling;
    go[e] = dout[(int64_t)b * lddo + h * dh + e];
  }
  __syncthreads();
  for (int t = wave; t < T; t += 4) {
    const float* kr = kv + ((int64_t)t * B + b) * ldkv + h * dh;
    const float* vr = kv + ((int64_t)t * B + b) * ldkv + v_off + h * dh;
    float acc = 0.f, accv = 0.f;
    for (int e = lane; e < dh; e += 64) {
      acc = fmaf(qs[e], kr[e], acc);
      accv = fmaf(go[e], vr[e], accv);
    }
    for (int o = 32; o >= 1; o >>= 1) {
      acc += __shfl_xor(acc, o, 64);
      accv += __shfl_xor(accv, o, 64);
    }
    if (lane == 0) {
      p[t] = acc;
      dp[t] = accv;
    }
  }
  __syncthreads();
  if (wave == 0) {
    float m = -INFINITY;
    for (int t = lane; t < T; t += 64) m = fmaxf(m, p[t]);
    m = wave_max(m);
    double s = 0.0;
    for (int t = lane; t < T; t += 64) {
      const float e = expf(p[t] - m);
      p[t] = e;
      s += (double)e;
    }
    s = wave_sum(s);
    const float inv = (float)(1.0 / s);
    double pd = 0.0;
    for (int t = lane; t < T; t += 64) {
      p[t] *= inv;
      pd += (double)p[t] * (double)dp[t];
    }
    pd = wave_sum(pd);
    if (lane == 0) red = pd;
  }
  __syncthreads();
  const double pdp = red;
  for (int t = tid; t < T; t += 256) dp[t] = (float)((double)p[t] * ((double)dp[t] - pdp));  // ds_t
  __syncthreads();
  // dK, dV rows (each (t, b, h) piece is written by this block only)
  for (int t = wave; t < T; t += 4) {
    float* dkr = dkv + ((int64_t)t * B + b) * lddkv + h * dh;
    float* dvr = dkv + ((int64_t)t * B + b) * lddkv + v_off + h * dh;
    const float ds = dp[t], pt = p[t];
    for (int e = lane; e < dh; e += 64) {
      dkr[e] = ds * qs[e];  // ds_t * scaling * q
      dvr[e] = pt * go[e];
    }
  }
  for (int e = lane; e < dh; e += 64) {
    float acc = 0.f;
    for (int t = wave; t < T; t += 4) acc = fmaf(dp[t], kv[((int64_t)t * B + b) * ldkv + h * dh + e], acc);
    pq[wave * dh + e] = acc;
  }
  __syncthreads();
  for (int e = tid; e < dh; e += 256)
    dq[(int64_t)b * lddq + h * dh + e] = scaling * ((pq[e] + pq[dh + e]) + (pq[2 * dh + e] + pq[3 * dh + e]));
}

__global__ __launch_bounds__(256) void combine_fwd_kernel(const float* __restrict__ y, const float* __restrict__ ds,
                                                          const float* __restrict__ text, const float* __restrict__ ref,
                                                          const float* __restrict__ based, int64_t B, int64_t d,
                                                          float* __restrict__ out) {
  const int64_t n = B * d;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float s = ds[i / d];
    out[i] = ((y[i] + s * text[i]) + (1.f - s) * ref[i]) + based[i];
  }
}

// one wave per row b: dtext = g ds, dref = g (1 - ds), dds = sum_j g (text - ref)
__global__ __launch_bounds__(256) void combine_bwd_kernel(const float* __restrict__ g, const float* __restrict__ ds,
                                                          const float* __restrict__ text, const float* __restrict__ ref,
                                                          int64_t B, int64_t d, float* __restrict__ dtext,
                                                          float* __restrict__ dref, float* __restrict__ dds) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float s = ds[b];
  double acc = 0.0;
  for (int64_t k = lane; k < d; k += 64) {
    const int64_t i = b * d + k;
    const float gv = g[i];
    if (dtext) dtext[i] = gv * s;
    if (dref) dref[i] = gv * (1.f - s);
    acc += (double)gv * (double)text[i] - (double)gv * (double)ref[i];
  }
  acc = wave_sum(acc);
  if (lane == 0 && dds) dds[b] = (float)acc;
}

__global__ __launch_bounds__(256) void pool_mean_bwd_kernel(const float* __restrict__ dy, int64_t B, int64_t T,
                                                            int64_t F, float* __restrict__ dx) {
  const int64_t n = B * T * F;
  const float inv = 1.f / (float)T;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / (T * F), f = i % F;
    dx[i] = dy[b * F + f] * inv;
  }
}

static unsigned grid_of(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192)); }

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_act_fwd(cmve_handle_t h, const float* x, int64_t n, int32_t kind, float* y) {
  CMVE_REQUIRE(h && (n == 0 || (x && y)) && n >= 0, "cmve_act_fwd: bad argument");
  CMVE_REQUIRE(kind >= 0 && kind <= 2, "cmve_act_fwd: unknown activation %d", kind);
  if (n == 0) return CMVE_OK;
  hipLaunchKernelGGL(act_fwd_kernel, dim3(grid_of(n)), dim3(256), 0, h->stream, x, n, kind, y);
  return check_launch("act_fwd");
}

extern "C" int cmve_act_bwd(cmve_handle_t h, const float* x, const float* dy, int64_t n, int32_t kind, float* dx) {
  CMVE_REQUIRE(h && (n == 0 || (x && dy && dx)) && n >= 0, "cmve_act_bwd: bad argument");
  CMVE_REQUIRE(kind >= 0 && kind <= 2, "cmve_act_bwd: unknown activation %d", kind);
  if (n == 0) return CMVE_OK;
  hipLaunchKernelGGL(act_bwd_kernel, dim3(grid_of(n)), dim3(256), 0, h->stream, x, dy, n, kind, dx);
  return check_launch("act_bwd");
}

extern "C" int cmve_layernorm_train_fwd(cmve_handle_t h, const float* x, int64_t ldx, int64_t n, int64_t d,
                                        const float* gamma, const float* beta, double eps, float* y, int64_t ldy,
                                        float* save_mean, float* save_rstd) {
  CMVE_REQUIRE(h && x && y && save_mean && save_rstd, "cmve_layernorm_train_fwd: NULL argument");
  CMVE_REQUIRE(n >= 0 && d > 0 && ldx >= d && ldy >= d, "cmve_layernorm_train_fwd: bad shape");
  if (n == 0) return CMVE_OK;
  hipLaunchKernelGGL(ln_train_fwd_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, h->stream, x, ldx, n, d, gamma,
                     beta, eps, y, ldy, save_mean, save_rstd);
  return check_launch("layernorm_train_fwd");
}

extern "C" int cmve_layernorm_bwd(cmve_handle_t h, const float* x, int64_t ldx, const float* dy, int64_t lddy,
                                  int64_t n, int64_t d, const float* gamma, const float* save_mean,
                                  const float* save_rstd, float* dx, int64_t lddx, float* dgamma, float* dbeta) {
  CMVE_REQUIRE(h && x && dy && save_mean && save_rstd, "cmve_layernorm_bwd: NULL argument");
  CMVE_REQUIRE(n >= 0 && d > 0 && ldx >= d && lddy >= d && (!dx || lddx >= d), "cmve_layernorm_bwd: bad shape");
  if (n == 0) return CMVE_OK;
  if (dx)
    hipLaunchKernelGGL(ln_bwd_dx_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, h->stream, x, ldx, dy, lddy, n,
                       d, gamma, save_mean, save_rstd, dx, lddx);
  if (dgamma || dbeta)
    hipLaunchKernelGGL(ln_bwd_param_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, h->stream, x, ldx, dy,
                       lddy, n, d, save_mean, save_rstd, dgamma, dbeta);
  return check_launch("layernorm_bwd");
}

extern "C" int cmve_mha_1q_bwd(cmve_handle_t h, const float* q, int64_t ldq, const float* kv, int64_t ldkv,
                               int64_t v_off, int32_t B, int32_t T, int32_t H, int32_t dh, const float* dout,
                               int64_t lddo, float* dq, int64_t lddq, float* dkv, int64_t lddkv) {
  CMVE_REQUIRE(h && q && kv && dout && dq && dkv, "cmve_mha_1q_bwd: NULL argument");
  const int64_t d = (int64_t)H * dh;
  CMVE_REQUIRE(B > 0 && T > 0 && H > 0 && dh > 0 && ldq >= d && lddo >= d && lddq >= d && v_off >= d &&
                   ldkv >= v_off + d && lddkv >= v_off + d,
               "cmve_mha_1q_bwd: bad shape");
  const size_t lds = sizeof(float) * (2 * (size_t)T + 6 * (size_t)dh);
  CMVE_REQUIRE(lds <= 64 * 1024, "cmve_mha_1q_bwd: T=%d, dh=%d exceed the LDS scratch", T, dh);
  hipLaunchKernelGGL(mha_1q_bwd_kernel, dim3((unsigned)B, (unsigned)H), dim3(256), lds, h->stream, q, ldq, kv, ldkv,
                     v_off, B, T, H, dh, dout, lddo, dq, lddq, dkv, lddkv);
  return check_launch("mha_1q_bwd");
}

extern "C" int cmve_combine_train_fwd(cmve_handle_t h, const float* y, const float* ds, const float* text,
                                      const float* ref, const float* based, int64_t B, int64_t d, float* out) {
  CMVE_REQUIRE(h && y && ds && text && ref && based && out && B >= 0 && d > 0, "cmve_combine_train_fwd: bad argument");
  if (B == 0) return CMVE_OK;
  hipLaunchKernelGGL(combine_fwd_kernel, dim3(grid_of(B * d)), dim3(256), 0, h->stream, y, ds, text, ref, based, B, d,
                     out);
  return check_launch("combine_train_fwd");
}

extern "C" int cmve_combine_train_bwd(cmve_handle_t h, const float* g, const float* ds, const float* text,
                                      const float* ref, int64_t B, int64_t d, float* dtext, float* dref, float* dds) {
  CMVE_REQUIRE(h && g && ds && text && ref && B >= 0 && d > 0, "cmve_combine_train_bwd: bad argument");
  if (B == 0) return CMVE_OK;
  hipLaunchKernelGGL(combine_bwd_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, h->stream, g, ds, text, ref, B,
                     d, dtext, dref, dds);
  return check_launch("combine_train_bwd");
}

extern "C" int cmve_pool_mean_bwd(cmve_handle_t h, const float* dy, int64_t B, int64_t T, int64_t F, float* dx) {
  CMVE_REQUIRE(h && dy && dx && B >= 0 && T > 0 && F > 0, "cmve_pool_mean_bwd: bad argument");
  if (B == 0) return CMVE_OK;
  hipLaunchKernelGGL(pool_mean_bwd_kernel, dim3(grid_of(B * T * F)), dim3(256), 0, h->stream, dy, B, T, F, dx);
  return check_launch("pool_mean_bwd");
}
