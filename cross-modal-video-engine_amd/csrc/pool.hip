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

// TSN feature-extraction head (MCT/mmaction/models/recognizers/recognizer2d.py:76-83): backbone maps
// x[B*S, C, HW] (NCHW, HW = H*W) -> AdaptiveAvgPool2d(1) per plane -> reshape (B, S, C) -> mean over S.
// Block = (64-channel group, video b), 4 waves; wave w takes segments s = w, w+4, ...: it copies the
// segment's contiguous [64 x HW] tile into its own LDS slab with float4 loads (row stride HW + 1: the
// per-channel reads below are conflict-free), then lane c sums plane c in hw order (fp32) and adds
// plane_sum / HW to its running segment sum.  The 4 wave partials are combined in wave order.
constexpr int TSN_CH = 64;
constexpr int TSN_MAX_HW = 128;  // LDS: 4 waves x 64 x (HW + 1) floats <= 129 KiB

__global__ __launch_bounds__(256) void tsn_pool_kernel(const float* __restrict__ x, int64_t S, int64_t C, int64_t HW,
                                                       float* __restrict__ out, int64_t ldo, int vec) {
  extern __shared__ float tsn_lds[];
  __shared__ float red[4][TSN_CH];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b = blockIdx.y, c0 = (int64_t)blockIdx.x * TSN_CH;
  const int64_t nch = C - c0 < TSN_CH ? C - c0 : TSN_CH;
  const int hw = (int)HW, tile = (int)(nch * HW);  // <= 64 * 128
  const float inv_hw = 1.f / (float)hw;
  // k -> (channel, position) without an integer divide: a float estimate, corrected by one step
  auto slab_at = [&](int k) {
    int ch = (int)((float)k * inv_hw);
    ch += (ch + 1) * hw <= k ? 1 : 0;
    ch -= ch * hw > k ? 1 : 0;
    return ch * (hw + 1) + (k - ch * hw);
  };
  float* slab = tsn_lds + w * TSN_CH * (hw + 1);
  float acc = 0.f;
  for (int64_t s = w; s < S; s += 4) {
    const float* src = x + ((b * S + s) * C + c0) * HW;
    if (vec) {  // src 16-byte aligned and tile % 4 == 0 (checked on the host)
      for (int i = lane * 4; i < tile; i += 256) {
        const f32x4_t v = *(const f32x4_t*)(src + i);
#pragma unroll
        for (int e = 0; e < 4; ++e) slab[slab_at(i + e)] = v[e];
      }
    } else {
      for (int k = lane; k < tile; k += 64) slab[slab_at(k)] = src[k];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes are done (the slab is wave-private)
    __builtin_amdgcn_wave_barrier();
    if (lane < nch) {
      float p = 0.f;
      for (int k = 0; k < hw; ++k) p += slab[lane * (hw + 1) + k];
      acc += p / (float)hw;
    }
    __builtin_amdgcn_wave_barrier();
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && lane < nch) {
    const float r = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    out[b * ldo + c0 + lane] = r / (float)S;
  }
}

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_tsn_pool(cmve_handle_t h, const float* x, int64_t B, int64_t S, int64_t C, int64_t HW, float* out,
                             int64_t ldo) {
  CMVE_REQUIRE(h && out && (B == 0 || x), "cmve_tsn_pool: NULL argument");
  CMVE_REQUIRE(B >= 0 && S > 0 && C > 0 && HW > 0 && ldo >= C, "cmve_tsn_pool: bad shape");
  CMVE_REQUIRE(HW <= TSN_MAX_HW, "cmve_tsn_pool: H*W = %lld > %d (pool the maps spatially first)", (long long)HW,
               TSN_MAX_HW);
  CMVE_REQUIRE(B <= 65535, "cmve_tsn_pool: B = %lld > 65535 videos per call", (long long)B);
  if (B == 0) return CMVE_OK;
  if (HW == 1) {  // maps already pooled spatially: [B, S, C] -> the MEAN_ALL temporal pool
    dim3 grid((unsigned)((C + 255) / 256), (unsigned)B);
    hipLaunchKernelGGL(pool_kernel<1>, grid, dim3(256), 0, h->stream, x, S * C, C, S, C, (const int32_t*)nullptr, out,
                       ldo);
    return check_launch("pool_kernel");
  }
  const int vec = ((uintptr_t)x % 16 == 0) && (C * HW) % 4 == 0 && (HW % 4 == 0 || C % TSN_CH == 0);
  const size_t lds = 4 * (size_t)TSN_CH * (size_t)(HW + 1) * sizeof(float);
  static const hipError_t attr_err =
      hipFuncSetAttribute((const void*)tsn_pool_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * TSN_CH *
                                                                                                      (TSN_MAX_HW + 1) *
                                                                                                      (int)sizeof(float));
  CMVE_HIP(attr_err);
  dim3 grid((unsigned)((C + TSN_CH - 1) / TSN_CH), (unsigned)B);
  hipLaunchKernelGGL(tsn_pool_kernel, grid, dim3(256), lds, h->stream, x, S, C, HW, out, ldo, vec);
  return check_launch("tsn_pool_kernel");
}

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
