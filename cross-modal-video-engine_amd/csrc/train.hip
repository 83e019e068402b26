// K11: training-step kernels for the projection heads, the pieces of
//   LINAS-engine/model.py:984-1004   train_emb, style 'GT': forward_emb -> TripletLoss ->
//                                    backward -> clip_grad_norm_ -> Adam step
// that are not GEMMs or the loss itself (those are K3 / gemm_f32 / K6 / K7):
//   BatchNorm1d training mode (batch statistics, running-stat update) forward + backward
//     (MFC.bn_1, model.py:83-85,111-112; torch BatchNorm1d semantics: biased variance normalises,
//     unbiased variance enters running_var, momentum 0.1)
//   column sums (Linear bias gradients), residual ReLU (model.py:104-109) and its mask gradient,
//   l2norm backward (model.py:35-40, no epsilon), counter-hash dropout (nn.Dropout, model.py:113-114),
//   clip_grad_norm_ (model.py:1001: fp64 sum of squares, deterministic order) and Adam
//   (model.py:593: torch.optim.Adam update order, fp32).
// All column statistics accumulate in fp64 in a fixed order (deterministic, run to run).
#include "cmve_internal.h"

#include <cmath>

namespace cmve {

constexpr int COLS = 16, RGRP = 16;  // column kernels: 16 columns x 16 row groups per 256-thread block

// block-wide sum over the 4 row groups of one column; all threads get the total
__device__ __forceinline__ double col_group_sum(double v, double (*red)[COLS]) {
  const int c = threadIdx.x % COLS, grp = threadIdx.x / COLS;
  red[grp][c] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < RGRP; ++k) s += red[k][c];  // fixed order
  __syncthreads();
  return s;
}

__global__ __launch_bounds__(256) void bn_train_fwd_kernel(const float* __restrict__ x, int64_t ldx, int64_t n,
                                                           int64_t d, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, double eps,
                                                           double momentum, float* __restrict__ rmean,
                                                           float* __restrict__ rvar, float* __restrict__ y,
                                                           int64_t ldy, float* __restrict__ smean,
                                                           float* __restrict__ sinvstd) {
  __shared__ double red[RGRP][COLS];
  const int64_t col = (int64_t)blockIdx.x * COLS + (threadIdx.x % COLS);
  const int grp = threadIdx.x / COLS;
  const bool ok = col < d;
  double s = 0.0;
  if (ok)
    for (int64_t r = grp; r < n; r += RGRP) s += (double)x[r * ldx + col];
  const double mean = col_group_sum(s, red) / (double)n;
  double q = 0.0;
  if (ok)
    for (int64_t r = grp; r < n; r += RGRP) {
      const double t = (double)x[r * ldx + col] - mean;
      q = fma(t, t, q);
    }
  const double var = col_group_sum(q, red) / (double)n;  // biased: what normalises the batch
  if (!ok) return;
  const double invstd = 1.0 / sqrt(var + eps);
  const double w = gamma ? (double)gamma[col] : 1.0, b = beta ? (double)beta[col] : 0.0;
  for (int64_t r = grp; r < n; r += RGRP) y[r * ldy + col] = (float)(((double)x[r * ldx + col] - mean) * invstd * w + b);
  if (grp == 0) {
    smean[col] = (float)mean;
    sinvstd[col] = (float)invstd;
    if (rmean) rmean[col] = (float)((1.0 - momentum) * (double)rmean[col] + momentum * mean);
    if (rvar) rvar[col] = (float)((1.0 - momentum) * (double)rvar[col] + momentum * var * (double)n / (double)(n - 1));
  }
}

// dx = gamma * invstd * (dy - mean(dy) - xhat * mean(dy * xhat)); dgamma = sum dy*xhat; dbeta = sum dy.
// The batch statistics are recomputed from x in fp64 rather than taken from the fp32 save_* of the
// forward: 1 - xhat^2 cancels badly for small batches (n = 2: dx ~ eps / (a^2 + eps)).
__global__ __launch_bounds__(256) void bn_train_bwd_kernel(const float* __restrict__ dy, int64_t lddy,
                                                           const float* __restrict__ x, int64_t ldx, int64_t n,
                                                           int64_t d, const float* __restrict__ gamma, double eps,
                                                           float* __restrict__ dx, int64_t lddx,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ double red[RGRP][COLS];
  const int64_t col = (int64_t)blockIdx.x * COLS + (threadIdx.x % COLS);
  const int grp = threadIdx.x / COLS;
  const bool ok = col < d;
  double s = 0.0;
  if (ok)
    for (int64_t r = grp; r < n; r += RGRP) s += (double)x[r * ldx + col];
  const double m = col_group_sum(s, red) / (double)n;
  double q = 0.0;
  if (ok)
    for (int64_t r = grp; r < n; r += RGRP) {
      const double t = (double)x[r * ldx + col] - m;
      q = fma(t, t, q);
    }
  const double is = 1.0 / sqrt(col_group_sum(q, red) / (double)n + eps);
  double sg = 0.0, sgx = 0.0;
  if (ok)
    for (int64_t r = grp; r < n; r += RGRP) {
      const double g = (double)dy[r * lddy + col];
      sg += g;
      sgx = fma(g, ((double)x[r * ldx + col] - m) * is, sgx);
    }
  sg = col_group_sum(sg, red);
  sgx = col_group_sum(sgx, red);
  if (!ok) return;
  const double w = gamma ? (double)gamma[col] : 1.0;
  if (dx) {
    const double mg = sg / (double)n, mgx = sgx / (double)n;
    for (int64_t r = grp; r < n; r += RGRP) {
      const double xh = ((double)x[r * ldx + col] - m) * is;
      dx[r * lddx + col] = (float)(((double)dy[r * lddy + col] - mg - xh * mgx) * is * w);
    }
  }
  if (grp == 0) {
    if (dgamma) dgamma[col] = (float)sgx;
    if (dbeta) dbeta[col] = (float)sg;
  }
}

__global__ __launch_bounds__(256) void col_sum_kernel(const float* __restrict__ x, int64_t ldx, int64_t n, int64_t d,
                                                      float* __restrict__ out) {
  __shared__ double red[RGRP][COLS];
  const int64_t col = (int64_t)blockIdx.x * COLS + (threadIdx.x % COLS);
  const int grp = threadIdx.x / COLS;
  double s = 0.0;
  if (col < d)
    for (int64_t r = grp; r < n; r += RGRP) s += (double)x[r * ldx + col];
  s = col_group_sum(s, red);
  if (col < d && grp == 0) out[col] = (float)s;
}

// out = resid + relu(z)  (model.py:104-109: features + relu(fc_k(features)))
__global__ __launch_bounds__(256) void resid_relu_kernel(const float* __restrict__ z, const float* __restrict__ resid,
                                                         int64_t n, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = z[i];
    out[i] = resid[i] + (v > 0.f ? v : 0.f);
  }
}

// dz = dout * (z > 0)
__global__ __launch_bounds__(256) void relu_grad_kernel(const float* __restrict__ z, const float* __restrict__ dout,
                                                        int64_t n, float* __restrict__ dz) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    dz[i] = z[i] > 0.f ? dout[i] : 0.f;
}

// y = x / ||x|| backward, wave per row: dx = dy / ||x|| - x * <x, dy> / ||x||^3  (fp64 per row)
__global__ __launch_bounds__(256) void l2norm_bwd_kernel(const float* __restrict__ x, int64_t ldx,
                                                         const float* __restrict__ dy, int64_t lddy, int64_t n,
                                                         int64_t d, float* __restrict__ dx, int64_t lddx) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const float* xr = x + r * ldx;
  const float* gr = dy + r * lddy;
  double ss = 0.0, xg = 0.0;
  for (int64_t k = lane; k < d; k += 64) {
    const double a = xr[k], g = gr[k];
    ss = fma(a, a, ss);
    xg = fma(a, g, xg);
  }
  ss = wave_sum(ss);
  xg = wave_sum(xg);
  const double inv = 1.0 / sqrt(ss);
  const double c = xg * inv * inv * inv;
  for (int64_t k = lane; k < d; k += 64) dx[r * lddx + k] = (float)((double)gr[k] * inv - (double)xr[k] * c);
}

// counter-based dropout hash (splitmix64 finaliser of seed + index): keep iff u >= p, u in [0, 1)
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void dropout_kernel(const float* __restrict__ x, int64_t n, float p, float scale,
                                                      uint64_t seed, uint64_t offset,
                                                      const int64_t* __restrict__ calls, float* __restrict__ y,
                                                      uint8_t* __restrict__ mask) {
  if (calls) offset += (uint64_t)calls[0] << 32;  // device-side stream position (graph replays advance it)
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint64_t h = mix64(seed + 0x9E3779B97F4A7C15ull * (offset + (uint64_t)i + 1));
    const float u = (float)(h >> 40) * (1.f / 16777216.f);
    const bool keep = u >= p;
    y[i] = keep ? x[i] * scale : 0.f;
    if (mask) mask[i] = keep;
  }
}

__global__ void counter_add_kernel(int64_t* __restrict__ c, int64_t by) { c[0] += by; }

__global__ __launch_bounds__(256) void mask_scale_kernel(const float* __restrict__ x, const uint8_t* __restrict__ mask,
                                                         int64_t n, float scale, float* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    y[i] = mask[i] ? x[i] * scale : 0.f;
}

// ---- clip_grad_norm_ + Adam over a list of tensors (multi-tensor launches, pointers by value) ----
constexpr int MT = 24;    // tensors per launch (kernel-argument table)
constexpr int MT_BPT = 128; // blocks per tensor (grid-stride inside a tensor; fixed partial layout)

struct MTList {
  float* p[MT];
  float* g[MT];
  float* m[MT];
  float* v[MT];
  int64_t n[MT];
  float step_size[MT];
  float bc2_sqrt[MT];
};

// partial[(base + t) * MT_BPT + b] = sum of g_t^2 over block b's grid-stride share (fp64, fixed order)
__global__ __launch_bounds__(256) void sumsq_multi_kernel(MTList L, int base, double* __restrict__ partial) {
  __shared__ double red[256];
  const int t = blockIdx.y;
  const float* __restrict__ x = L.g[t];
  const int64_t n = L.n[t];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)MT_BPT * 256) {
    const double v = x[i];
    s = fma(v, v, s);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[(int64_t)(base + t) * MT_BPT + blockIdx.x] = red[0];
}

// total = sqrt(sum partial); coef = min(1, max_norm / (total + 1e-6))   (torch clip_grad_norm_)
__global__ __launch_bounds__(256) void clip_coef_kernel(const double* __restrict__ partial, int64_t count,
                                                        double max_norm, float* __restrict__ coef,
                                                        float* __restrict__ total) {
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < count; i += 256) s += partial[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float tn = (float)sqrt(red[0]);
    const float c = (float)max_norm / (tn + 1e-6f);
    if (coef) coef[0] = c < 1.f ? c : 1.f;
    if (total) total[0] = tn;
  }
}

__global__ __launch_bounds__(256) void scale_multi_kernel(MTList L, const float* __restrict__ coef) {
  const int t = blockIdx.y;
  float* __restrict__ x = L.g[t];
  const int64_t n = L.n[t];
  const float c = coef[0];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) x[i] *= c;
}

// torch.optim.Adam (single-tensor order, fp32): [g *= coef, written back like clip_grad_norm_];
// g += wd * p; m = lerp(m, g, 1 - b1); v = b2 * v + (1 - b2) * g * g;
// p -= step_size * m / (sqrt(v) / bc2_sqrt + eps)
__global__ __launch_bounds__(256) void adam_multi_kernel(MTList L, float b1, float b2, float eps, float wd,
                                                         const float* __restrict__ grad_scale,
                                                         const int64_t* __restrict__ dev_step, double lr, double b1d,
                                                         double b2d) {
  const int t = blockIdx.y;
  float* __restrict__ p = L.p[t];
  float* __restrict__ g = L.g[t];
  float* __restrict__ m = L.m[t];
  float* __restrict__ v = L.v[t];
  const int64_t n = L.n[t];
  float step_size = L.step_size[t], bc2s = L.bc2_sqrt[t];
  if (dev_step) {  // capturable: the step count lives on the device (same fp64 scalar formulas as the host)
    const double st = (double)dev_step[0];
    step_size = (float)(lr / (1.0 - pow(b1d, st)));
    bc2s = (float)sqrt(1.0 - pow(b2d, st));
  }
  const float w = 1.f - b1;
  const float c = grad_scale ? grad_scale[0] : 1.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float gi = g[i];
    if (grad_scale) {
      gi *= c;
      g[i] = gi;
    }
    if (wd != 0.f) gi = gi + wd * p[i];
    const float mi = m[i], mo = mi + w * (gi - mi);  // lerp, weight < 0.5 branch
    const float vo = v[i] * b2 + (1.f - b2) * gi * gi;
    m[i] = mo;
    v[i] = vo;
    const float denom = sqrtf(vo) / bc2s + eps;
    p[i] = p[i] + (-step_size) * (mo / denom);
  }
}

inline unsigned ew_grid(int64_t n) { return (unsigned)std::min<int64_t>((n + 255) / 256, 4096); }
inline unsigned col_grid(int64_t d) { return (unsigned)((d + COLS - 1) / COLS); }

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_bn_train_fwd(cmve_handle_t h, const float* x, int64_t ldx, int64_t n, int64_t d,
                                 const float* gamma, const float* beta, double eps, double momentum,
                                 float* running_mean, float* running_var, float* y, int64_t ldy, float* save_mean,
                                 float* save_invstd) {
  CMVE_REQUIRE(h && x && y && save_mean && save_invstd, "cmve_bn_train_fwd: NULL argument");
  CMVE_REQUIRE(n > 1, "cmve_bn_train_fwd: expected more than 1 value per channel when training, got n=%lld",
               (long long)n);
  CMVE_REQUIRE(d > 0 && ldx >= d && ldy >= d, "cmve_bn_train_fwd: bad shape");
  hipLaunchKernelGGL(bn_train_fwd_kernel, dim3(col_grid(d)), dim3(256), 0, h->stream, x, ldx, n, d, gamma, beta, eps,
                     momentum, running_mean, running_var, y, ldy, save_mean, save_invstd);
  return check_launch("bn_train_fwd");
}

extern "C" int cmve_bn_train_bwd(cmve_handle_t h, const float* dy, int64_t lddy, const float* x, int64_t ldx,
                                 int64_t n, int64_t d, const float* gamma, double eps, float* dx, int64_t lddx,
                                 float* dgamma, float* dbeta) {
  CMVE_REQUIRE(h && dy && x, "cmve_bn_train_bwd: NULL argument");
  CMVE_REQUIRE(n > 1 && d > 0 && lddy >= d && ldx >= d && (!dx || lddx >= d), "cmve_bn_train_bwd: bad shape");
  hipLaunchKernelGGL(bn_train_bwd_kernel, dim3(col_grid(d)), dim3(256), 0, h->stream, dy, lddy, x, ldx, n, d, gamma,
                     eps, dx, lddx, dgamma, dbeta);
  return check_launch("bn_train_bwd");
}

extern "C" int cmve_col_sum(cmve_handle_t h, const float* x, int64_t ldx, int64_t n, int64_t d, float* out) {
  CMVE_REQUIRE(h && x && out, "cmve_col_sum: NULL argument");
  CMVE_REQUIRE(n >= 0 && d > 0 && ldx >= d, "cmve_col_sum: bad shape");
  hipLaunchKernelGGL(col_sum_kernel, dim3(col_grid(d)), dim3(256), 0, h->stream, x, ldx, n, d, out);
  return check_launch("col_sum");
}

extern "C" int cmve_resid_relu(cmve_handle_t h, const float* z, const float* resid, int64_t n, float* out) {
  CMVE_REQUIRE(h && z && resid && out && n >= 0, "cmve_resid_relu: bad argument");
  if (n == 0) return CMVE_OK;
  hipLaunchKernelGGL(resid_relu_kernel, dim3(ew_grid(n)), dim3(256), 0, h->stream, z, resid, n, out);
  return check_launch("resid_relu");
}

extern "C" int cmve_relu_grad(cmve_handle_t h, const float* z, const float* dout, int64_t n, float* dz) {
  CMVE_REQUIRE(h && z && dout && dz && n >= 0, "cmve_relu_grad: bad argument");
  if (n == 0) return CMVE_OK;
  hipLaunchKernelGGL(relu_grad_kernel, dim3(ew_grid(n)), dim3(256), 0, h->stream, z, dout, n, dz);
  return check_launch("relu_grad");
}

extern "C" int cmve_l2norm_bwd(cmve_handle_t h, const float* x, int64_t ldx, const float* dy, int64_t lddy, int64_t n,
                               int64_t d, float* dx, int64_t lddx) {
  CMVE_REQUIRE(h && x && dy && dx, "cmve_l2norm_bwd: NULL argument");
  CMVE_REQUIRE(n >= 0 && d > 0 && ldx >= d && lddy >= d && lddx >= d, "cmve_l2norm_bwd: bad shape");
  if (n == 0) return CMVE_OK;
  hipLaunchKernelGGL(l2norm_bwd_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, h->stream, x, ldx, dy, lddy, n, d,
                     dx, lddx);
  return check_launch("l2norm_bwd");
}

extern "C" int cmve_dropout(cmve_handle_t h, const float* x, int64_t n, float p, uint64_t seed, uint64_t offset,
                            float* y, uint8_t* mask, int64_t* call_counter) {
  CMVE_REQUIRE(h && x && y && n >= 0, "cmve_dropout: bad argument");
  CMVE_REQUIRE(p >= 0.f && p < 1.f, "cmve_dropout: p must be in [0, 1), got %g", (double)p);
  if (n > 0)
    hipLaunchKernelGGL(dropout_kernel, dim3(ew_grid(n)), dim3(256), 0, h->stream, x, n, p, 1.f / (1.f - p), seed,
                       offset, call_counter, y, mask);
  if (call_counter) hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(1), 0, h->stream, call_counter, (int64_t)1);
  return check_launch("dropout");
}

extern "C" int cmve_mask_scale(cmve_handle_t h, const float* x, const uint8_t* mask, int64_t n, float scale, float* y) {
  CMVE_REQUIRE(h && x && mask && y && n >= 0, "cmve_mask_scale: bad argument");
  if (n == 0) return CMVE_OK;
  hipLaunchKernelGGL(mask_scale_kernel, dim3(ew_grid(n)), dim3(256), 0, h->stream, x, mask, n, scale, y);
  return check_launch("mask_scale");
}

static unsigned mt_blocks(const MTList& L, int cnt) {
  int64_t mx = 1;
  for (int i = 0; i < cnt; ++i) mx = std::max(mx, L.n[i]);
  return (unsigned)std::min<int64_t>((mx + 1023) / 1024, 256);
}

extern "C" int cmve_grad_norm_multi(cmve_handle_t h, int32_t n, float* const* grads, const int64_t* numels,
                                    double max_norm, float* coef, float* total_norm) {
  CMVE_REQUIRE(h && n >= 0 && (n == 0 || (grads && numels)) && (coef || total_norm),
               "cmve_grad_norm_multi: bad argument");
  const int64_t count = (int64_t)std::max(n, 1) * MT_BPT;
  const int rc = ensure_scratch(h, (size_t)count * sizeof(double));
  if (rc != CMVE_OK) return rc;
  double* partial = (double*)h->scratch;
  if (n == 0) CMVE_HIP(hipMemsetAsync(partial, 0, sizeof(double) * MT_BPT, h->stream));
  for (int base = 0; base < n; base += MT) {
    MTList L = {};
    const int cnt = std::min(MT, n - base);
    for (int i = 0; i < cnt; ++i) {
      CMVE_REQUIRE(grads[base + i] && numels[base + i] >= 0, "cmve_grad_norm_multi: tensor %d", base + i);
      L.g[i] = grads[base + i];
      L.n[i] = numels[base + i];
    }
    hipLaunchKernelGGL(sumsq_multi_kernel, dim3(MT_BPT, cnt), dim3(256), 0, h->stream, L, base, partial);
  }
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(256), 0, h->stream, partial, count, max_norm, coef, total_norm);
  return check_launch("grad_norm_multi");
}

extern "C" int cmve_scale_multi(cmve_handle_t h, int32_t n, float* const* xs, const int64_t* numels, const float* coef) {
  CMVE_REQUIRE(h && coef && n >= 0 && (n == 0 || (xs && numels)), "cmve_scale_multi: bad argument");
  for (int base = 0; base < n; base += MT) {
    MTList L = {};
    const int cnt = std::min(MT, n - base);
    for (int i = 0; i < cnt; ++i) {
      CMVE_REQUIRE(xs[base + i] && numels[base + i] >= 0, "cmve_scale_multi: tensor %d", base + i);
      L.g[i] = xs[base + i];
      L.n[i] = numels[base + i];
    }
    hipLaunchKernelGGL(scale_multi_kernel, dim3(mt_blocks(L, cnt), cnt), dim3(256), 0, h->stream, L, coef);
  }
  return check_launch("scale_multi");
}

extern "C" int cmve_adam_multi(cmve_handle_t h, int32_t n, float* const* params, float* const* grads,
                               float* const* exp_avgs, float* const* exp_avg_sqs, const int64_t* numels,
                               const int64_t* steps, double lr, double beta1, double beta2, double eps,
                               double weight_decay, const float* grad_scale, int64_t* dev_step) {
  CMVE_REQUIRE(h && n >= 0 && (n == 0 || (params && grads && exp_avgs && exp_avg_sqs && numels && (steps || dev_step))),
               "cmve_adam_multi: bad argument");
  if (dev_step) hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(1), 0, h->stream, dev_step, (int64_t)1);
  for (int base = 0; base < n; base += MT) {
    MTList L = {};
    const int cnt = std::min(MT, n - base);
    for (int i = 0; i < cnt; ++i) {
      const int k = base + i;
      CMVE_REQUIRE(params[k] && grads[k] && exp_avgs[k] && exp_avg_sqs[k] && numels[k] >= 0 && (dev_step || steps[k] >= 1),
                   "cmve_adam_multi: tensor %d (steps count from 1)", k);
      L.p[i] = params[k];
      L.g[i] = grads[k];
      L.m[i] = exp_avgs[k];
      L.v[i] = exp_avg_sqs[k];
      L.n[i] = numels[k];
      if (!dev_step) {  // host-side scalars exactly as torch.optim.Adam forms them (Python floats)
        const double bc1 = 1.0 - std::pow(beta1, (double)steps[k]);
        const double bc2 = 1.0 - std::pow(beta2, (double)steps[k]);
        L.step_size[i] = (float)(lr / bc1);
        L.bc2_sqrt[i] = (float)std::sqrt(bc2);
      }
    }
    hipLaunchKernelGGL(adam_multi_kernel, dim3(mt_blocks(L, cnt), cnt), dim3(256), 0, h->stream, L, (float)beta1,
                       (float)beta2, (float)eps, (float)weight_decay, grad_scale, (const int64_t*)dev_step, lr, beta1,
                       beta2);
  }
  return check_launch("adam_multi");
}
