// K2: temporal pooling over frames (HBM-bound; float4 loads, one thread per 4 features,
// sequential fp32 accumulation over t like a per-column loop).
//
//   cmve_collate_frames  -- LINAS-engine/util/tag_data_provider.py:91-109 (collate_frame):
//       videos[b, :min(64,T_b), :] = frames_b[:min(64,T_b)], zero padding to T_max,
//       origin[b] = mean over ALL T_b frames (tag_data_provider.py:104), mask[b, t] = t < min(64,T_b)
//   cmve_temporal_pool modes:
//       MEAN_VALID       mean over t < len[b]      LINAS-engine/model.py:152-156 (gru_pool='mean')
//       MEAN_ALL         mean over all T           MultiFusion/src/combiner.py:140-143 (time_process),
//                                                  MCT/mmaction/models/recognizers/recognizer2d.py:76-83 (TSN)
//       MAX_MASKED_ZERO  max_t x[t] * mask[t]      LINAS-engine/model.py:157-158 (masked steps contribute 0)
//       MAX_ALL          max over all T            LINAS-engine/model.py:163-166 (max_pool1d over padded length)
//   cmve_adaptive_avg_pool2d -- F.adaptive_avg_pool2d of the reference video's middle tokens
//       (MultiFusion/src/inference.py:58-59: [1, T, 18*18, C] -> [1, T, 16, D]); windows
//       [floor(i*H/OH), ceil((i+1)*H/OH)) x [floor(j*W/OW), ceil((j+1)*W/OW)) as ATen defines them.
#include "cmve_internal.h"

namespace cmve {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void collate_kernel(const float* __restrict__ frames, int64_t ldf,
                                                      const int64_t* __restrict__ off, int64_t F, int max_len,
                                                      int t_max, float* __restrict__ videos, float* __restrict__ origin,
                                                      float* __restrict__ mask) {
  const int64_t b = blockIdx.y;
  const int64_t f0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t r0 = off[b], T = off[b + 1] - off[b];
  const int keep = (int)(T < max_len ? T : max_len);
  if (blockIdx.x == 0)
    for (int t = threadIdx.x; t < t_max; t += 256) mask[b * t_max + t] = t < keep ? 1.f : 0.f;
  if (f0 >= F) return;
  const bool vec = (f0 + 4 <= F) && ((ldf & 3) == 0) && ((F & 3) == 0);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int64_t t = 0; t < T; ++t) {
    const float* src = frames + (r0 + t) * ldf + f0;
    float v[4];
    if (vec) {
      const f32x4_t x = *(const f32x4_t*)src;
      v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
    } else {
      for (int e = 0; e < 4; ++e) v[e] = (f0 + e < F) ? src[e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] += v[e];
    if (t < keep) {
      float* dst = videos + (b * t_max + t) * F + f0;
      for (int e = 0; e < 4; ++e)
        if (f0 + e < F) dst[e] = v[e];
    }
  }
  for (int t = keep; t < t_max; ++t) {
    float* dst = videos + (b * t_max + t) * F + f0;
    for (int e = 0; e < 4; ++e)
      if (f0 + e < F) dst[e] = 0.f;
  }
  for (int e = 0; e < 4; ++e)
    if (f0 + e < F) origin[b * F + f0 + e] = T > 0 ? acc[e] / (float)T : NAN;
}

// block = (256-float chunk of F, video b); 4 waves split the frames (t = w, w + 4, ...), each lane owns
// 4 consecutive features (float4); the 4 wave partials are combined through LDS in fixed wave order.
template <int MODE>
__global__ __launch_bounds__(256) void pool_kernel(const float* __restrict__ x, int64_t sb, int64_t st, int64_t T,
                                                   int64_t F, const int32_t* __restrict__ lengths,
                                                   float* __restrict__ out, int64_t ldo) {
  __shared__ float red[4][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b = blockIdx.y;
  const int64_t f0 = (int64_t)blockIdx.x * 256 + lane * 4;
  const int64_t len = lengths ? (int64_t)lengths[b] : T;
  const int64_t tend = (MODE == 0) ? (len < T ? len : T) : T;  // MEAN_VALID stops at len
  const bool vec = (f0 + 4 <= F) && ((st & 3) == 0) && ((sb & 3) == 0) && ((F & 3) == 0);
  float acc[4];
  for (int e = 0; e < 4; ++e) acc[e] = (MODE >= 2) ? -INFINITY : 0.f;
  if (f0 < F) {
#pragma unroll 4
    for (int64_t t = w; t < tend; t += 4) {
      const float* src = x + b * sb + t * st + f0;
      float v[4];
      if (vec) {
        const f32x4_t q = *(const f32x4_t*)src;
        v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
      } else {
        for (int e = 0; e < 4; ++e) v[e] = (f0 + e < F) ? src[e] : 0.f;
      }
      if (MODE == 2) {  // masked steps contribute x * 0
        const float m = t < len ? 1.f : 0.f;
        for (int e = 0; e < 4; ++e) v[e] *= m;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (MODE <= 1) acc[e] += v[e];
        else acc[e] = (v[e] > acc[e] || v[e] != v[e]) ? v[e] : acc[e];  // torch.max propagates NaN
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) red[w][lane * 4 + e] = acc[e];
  __syncthreads();
  if (w != 0 || f0 >= F) return;
  for (int e = 0; e < 4; ++e) {
    if (f0 + e >= F) break;
    float r = red[0][lane * 4 + e];
    for (int k = 1; k < 4; ++k) {
      const float q = red[k][lane * 4 + e];
      if (MODE <= 1) r += q;
      else r = (q > r || q != q) ? q : r;
    }
    if (MODE == 0) r = tend > 0 ? r / (float)tend : NAN;
    if (MODE == 1) r = r / (float)T;
    out[b * ldo + f0 + e] = r;
  }
}

// block = (output row i, plane p): the window's input rows are summed per column into LDS (one
// coalesced pass over the rows, each input row read by at most two blocks), then each thread sums
// the column window of its output columns and divides by the window area.
__global__ __launch_bounds__(256) void adaptive_avg_kernel(const float* __restrict__ x, int64_t H, int64_t W,
                                                           int64_t sp, int64_t sh, int64_t OH, int64_t OW,
                                                           float* __restrict__ out) {
  extern __shared__ float colsum[];
  const int64_t i = blockIdx.x, p = blockIdx.y;
  const int64_t hs = (i * H) / OH, he = ((i + 1) * H + OH - 1) / OH;
  const float* src = x + p * sp;
  for (int64_t c = threadIdx.x; c < W; c += 256) {
    float s = 0.f;
    for (int64_t r = hs; r < he; ++r) s += src[r * sh + c];
    colsum[c] = s;
  }
  __syncthreads();
  const float rows = (float)(he - hs);
  for (int64_t j = threadIdx.x; j < OW; j += 256) {
    const int64_t ws = (j * W) / OW, we = ((j + 1) * W + OW - 1) / OW;
    float s = 0.f;
    for (int64_t c = ws; c < we; ++c) s += colsum[c];
    out[(p * OH + i) * OW + j] = s / (rows * (float)(we - ws));
  }
}

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_adaptive_avg_pool2d(cmve_handle_t h, const float* x, int64_t P, int64_t H, int64_t W,
                                        int64_t sp, int64_t sh, int64_t OH, int64_t OW, float* out) {
  CMVE_REQUIRE(h && x && out, "cmve_adaptive_avg_pool2d: NULL argument");
  CMVE_REQUIRE(P >= 0 && H > 0 && W > 0 && OH > 0 && OW > 0 && sh >= W && sp >= (H - 1) * sh + W,
               "cmve_adaptive_avg_pool2d: bad shape");
  CMVE_REQUIRE(W * (int64_t)sizeof(float) <= 64 * 1024, "cmve_adaptive_avg_pool2d: W=%lld exceeds the LDS row",
               (long long)W);
  CMVE_REQUIRE(OH <= 65535 * 1024 && P <= 65535, "cmve_adaptive_avg_pool2d: grid too large");
  if (P == 0) return CMVE_OK;
  hipLaunchKernelGGL(adaptive_avg_kernel, dim3((unsigned)OH, (unsigned)P), dim3(256), W * sizeof(float), h->stream,
                     x, H, W, sp, sh, OH, OW, out);
  return check_launch("adaptive_avg_kernel");
}

extern "C" int cmve_collate_frames(cmve_handle_t h, const float* frames, int64_t ldf, const int64_t* offsets,
                                   int64_t B, int64_t F, int32_t max_len, int32_t t_max, float* videos,
                                   float* origin, float* mask) {
  CMVE_REQUIRE(h && offsets && videos && origin && mask, "cmve_collate_frames: NULL argument");
  CMVE_REQUIRE(B >= 0 && F > 0 && ldf >= F && max_len > 0 && t_max >= 0, "cmve_collate_frames: bad shape");
  CMVE_REQUIRE(B == 0 || frames, "cmve_collate_frames: frames is NULL");
  if (B == 0) return CMVE_OK;
  dim3 grid((unsigned)((F + 1023) / 1024), (unsigned)B);
  hipLaunchKernelGGL(collate_kernel, grid, dim3(256), 0, h->stream, frames, ldf, offsets, F, max_len, t_max, videos,
                     origin, mask);
  return check_launch("collate_kernel");
}

extern "C" int cmve_temporal_pool(cmve_handle_t h, const float* x, int64_t stride_b, int64_t stride_t, int64_t B,
                                  int64_t T, int64_t F, const int32_t* lengths, int32_t mode, float* out,
                                  int64_t ldo) {
  CMVE_REQUIRE(h && x && out, "cmve_temporal_pool: NULL argument");
  CMVE_REQUIRE(B >= 0 && T > 0 && F > 0 && ldo >= F, "cmve_temporal_pool: bad shape");
  CMVE_REQUIRE(mode >= 0 && mode <= 3, "cmve_temporal_pool: unknown mode %d", mode);
  CMVE_REQUIRE(!(mode == 0 || mode == 2) || lengths, "cmve_temporal_pool: this mode needs lengths");
  if (B == 0) return CMVE_OK;
  dim3 grid((unsigned)((F + 255) / 256), (unsigned)B);
#define POOL(M) \
  hipLaunchKernelGGL(pool_kernel<M>, grid, dim3(256), 0, h->stream, x, stride_b, stride_t, T, F, lengths, out, ldo)
  switch (mode) {
    case 0: POOL(0); break;
    case 1: POOL(1); break;
    case 2: POOL(2); break;
    default: POOL(3); break;
  }
#undef POOL
  return check_launch("pool_kernel");
}
