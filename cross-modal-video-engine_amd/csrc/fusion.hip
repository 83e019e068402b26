// K8 / K9: the non-GEMM pieces of MultiFusion's Combiner.combine_features
// (MultiFusion/src/combiner.py:19-43,146-180).  Its GEMMs (conv1x1, q/kv in-projections,
// out_proj, MLP, projection / combiner / dynamic-scalar / output layers) run on cmve_linear.
//
//   cmve_layernorm      LayerNorm (fp32 subclass, combiner.py:11-17), eps 1e-5; fp64 statistics
//   cmve_mha_1q         nn.MultiheadAttention(d, H) with ONE query per batch element and T keys,
//                       key t of batch b at row t*B + b of the projected K/V matrix -- exactly the
//                       raw p_s_m.reshape(l*f, b, d) of combiner.py:164-165 (mixes batch rows)
//   cmve_fuse_combine   out = normalize( y + ds*text + (1-ds)*ref + relu(based) )   (combiner.py:166,178-180)
#include "cmve_internal.h"

namespace cmve {

__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int64_t ldx, int64_t n,
                                                        int64_t d, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, double eps,
                                                        float* __restrict__ y, int64_t ldy) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const float* xr = x + row * ldx;
  if (d <= 1024) {  // the row read once into registers (16 per lane); same per-lane order as below
    float v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = (lane + 64 * m < d) ? xr[lane + 64 * m] : 0.f;
    double s = 0.0;
#pragma unroll
    for (int m = 0; m < 16; ++m)
      if (lane + 64 * m < d) s += (double)v[m];
    const double mean = wave_sum(s) / (double)d;
    double q = 0.0;
#pragma unroll
    for (int m = 0; m < 16; ++m)
      if (lane + 64 * m < d) {
        const double c = (double)v[m] - mean;
        q = fma(c, c, q);
      }
    const double rstd = 1.0 / sqrt(wave_sum(q) / (double)d + eps);
    float* yr = y + row * ldy;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int64_t k = lane + 64 * m;
      if (k < d) {
        const double c = ((double)v[m] - mean) * rstd;
        yr[k] = (float)(c * (double)(gamma ? gamma[k] : 1.f) + (double)(beta ? beta[k] : 0.f));
      }
    }
    return;
  }
  double s = 0.0;
  for (int64_t k = lane; k < d; k += 64) s += (double)xr[k];
  const double mean = wave_sum(s) / (double)d;
  double v = 0.0;
  for (int64_t k = lane; k < d; k += 64) {
    const double c = (double)xr[k] - mean;
    v = fma(c, c, v);
  }
  const double rstd = 1.0 / sqrt(wave_sum(v) / (double)d + eps);  // biased variance, as nn.LayerNorm
  float* yr = y + row * ldy;
  for (int64_t k = lane; k < d; k += 64) {
    const double c = ((double)xr[k] - mean) * rstd;
    yr[k] = (float)(c * (double)(gamma ? gamma[k] : 1.f) + (double)(beta ? beta[k] : 0.f));
  }
}

// block per (batch b, head h); 4 waves split the T keys, softmax in fp32 with fp64 sums
__global__ __launch_bounds__(256) void mha_1q_kernel(const float* __restrict__ q, int64_t ldq,
                                                     const float* __restrict__ kv, int64_t ldkv, int64_t v_off, int B,
                                                     int T, int H, int dh, float* __restrict__ out, int64_t ldo) {
  extern __shared__ float sh[];  // scores[T] + qs[dh] + partial out [4][dh]
  float* sc = sh;
  float* qs = sc + T;
  float* po = qs + dh;
  const int b = blockIdx.x, h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float scaling = 1.0f / sqrtf((float)dh);  // F.multi_head_attention_forward: q * head_dim^-0.5
  for (int e = tid; e < dh; e += 256) qs[e] = q[(int64_t)b * ldq + h * dh + e] * scaling;
  __syncthreads();
  for (int t = wave; t < T; t += 4) {
    const float* kr = kv + ((int64_t)t * B + b) * ldkv + h * dh;
    float acc = 0.f;
    for (int e = lane; e < dh; e += 64) acc = fmaf(qs[e], kr[e], acc);
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) sc[t] = acc;
  }
  __syncthreads();
  if (wave == 0) {  // softmax over T
    float m = -INFINITY;
    for (int t = lane; t < T; t += 64) m = fmaxf(m, sc[t]);
    m = wave_max(m);
    double s = 0.0;
    for (int t = lane; t < T; t += 64) {
      const float p = expf(sc[t] - m);
      sc[t] = p;
      s += (double)p;
    }
    s = wave_sum(s);
    const float inv = (float)(1.0 / s);
    for (int t = lane; t < T; t += 64) sc[t] *= inv;
  }
  __syncthreads();
  for (int e = lane; e < dh; e += 64) {
    float acc = 0.f;
    for (int t = wave; t < T; t += 4) acc = fmaf(sc[t], kv[((int64_t)t * B + b) * ldkv + v_off + h * dh + e], acc);
    po[wave * dh + e] = acc;
  }
  __syncthreads();
  for (int e = tid; e < dh; e += 256)
    out[(int64_t)b * ldo + h * dh + e] = (po[e] + po[dh + e]) + (po[2 * dh + e] + po[3 * dh + e]);
}

// out = normalize( ((y + ds*text) + (1-ds)*ref) + based , eps )
__global__ __launch_bounds__(256) void fuse_combine_kernel(const float* __restrict__ y, const float* __restrict__ ds,
                                                           const float* __restrict__ text,
                                                           const float* __restrict__ ref,
                                                           const float* __restrict__ based, int64_t n, int64_t d,
                                                           double eps, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const float s = ds[row];
  const float s1 = 1.f - s;
  double ss = 0.0;
  for (int64_t k = lane; k < d; k += 64) {
    const int64_t i = row * d + k;
    const float v = ((y[i] + s * text[i]) + s1 * ref[i]) + fmaxf(based[i], 0.f);  // based = relu(block out)
    out[i] = v;
    ss = fma((double)v, (double)v, ss);
  }
  const double den = fmax(sqrt(wave_sum(ss)), eps);
  for (int64_t k = lane; k < d; k += 64) {
    const int64_t i = row * d + k;
    out[i] = (float)((double)out[i] / den);
  }
}

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_layernorm(cmve_handle_t h, const float* x, int64_t ldx, int64_t n, int64_t d, const float* gamma,
                              const float* beta, double eps, float* y, int64_t ldy) {
  CMVE_REQUIRE(h && x && y, "cmve_layernorm: NULL argument");
  CMVE_REQUIRE(n >= 0 && d > 0 && ldx >= d && ldy >= d, "cmve_layernorm: bad shape");
  if (n == 0) return CMVE_OK;
  hipLaunchKernelGGL(layernorm_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, h->stream, x, ldx, n, d, gamma,
                     beta, eps, y, ldy);
  return check_launch("layernorm");
}

extern "C" int cmve_mha_1q(cmve_handle_t h, const float* q, int64_t ldq, const float* kv, int64_t ldkv, int64_t v_off,
                           int32_t B, int32_t T, int32_t H, int32_t dh, float* out, int64_t ldo) {
  CMVE_REQUIRE(h && q && kv && out, "cmve_mha_1q: NULL argument");
  CMVE_REQUIRE(B > 0 && T > 0 && H > 0 && dh > 0 && ldq >= (int64_t)H * dh && ldo >= (int64_t)H * dh,
               "cmve_mha_1q: bad shape");
  const size_t lds = sizeof(float) * ((size_t)T + dh + 4 * (size_t)dh);
  CMVE_REQUIRE(lds <= 64 * 1024, "cmve_mha_1q: T/dh too large for one block");
  hipLaunchKernelGGL(mha_1q_kernel, dim3((unsigned)B, (unsigned)H), dim3(256), lds, h->stream, q, ldq, kv, ldkv, v_off,
                     B, T, H, dh, out, ldo);
  return check_launch("mha_1q");
}

extern "C" int cmve_fuse_combine(cmve_handle_t h, const float* y, const float* ds, const float* text, const float* ref,
                                 const float* based, int64_t n, int64_t d, double eps, float* out) {
  CMVE_REQUIRE(h && y && ds && text && ref && based && out, "cmve_fuse_combine: NULL argument");
  if (n == 0) return CMVE_OK;
  hipLaunchKernelGGL(fuse_combine_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, h->stream, y, ds, text, ref,
                     based, n, d, eps, out);
  return check_launch("fuse_combine");
}
