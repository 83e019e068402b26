// K8 / K9: the non-GEMM pieces of MultiFusion's Combiner.combine_features
// (MultiFusion/src/combiner.py:19-43,146-180).  Its GEMMs (conv1x1, q/kv in-projections,
// out_proj, MLP, projection / combiner / dynamic-scalar / output layers) run on cmve_linear.
//
//   cmve_layernorm      LayerNorm (fp32 subclass, combiner.py:11-17), eps 1e-5; fp64 statistics
//   cmve_mha_1q         nn.MultiheadAttention(d, H) with ONE query per batch element and T keys,
//                       key t of batch b at row t*B + b of the projected K/V matrix -- exactly the
//                       raw p_s_m.reshape(l*f, b, d) of combiner.py:164-165 (mixes batch rows)
//   cmve_fuse_combine   out = normalize( y + ds*text + (1-ds)*ref + relu(based) )   (combiner.py:166,178-180)
//   cmve_transpose_blocks / cmve_pack_tblocks / cmve_layernorm_pack: the raw reshapes around the
//                       conv1x1 (combiner.py:159: mid.reshape(b*f, -1, 4, 4) -> its GEMM rows are the
//                       COLUMNS of each [640, 16] block; the output goes back through .reshape) as
//                       LDS-tiled block transposes, the transpose of the conv input fused with the
//                       split-bf16 packing of the GEMM operand, and the key LayerNorm fused with the
//                       packing of the K/V in-projection's operand (no fp32 round trip)
#include "cmve_internal.h"

namespace cmve {

// One row of LayerNorm held in registers as float4 runs (d <= 1024, d % 4 == 0, 16-byte aligned
// rows): lane owns elements 4j .. 4j+3 for j = lane + 64 m.  fp64 statistics (biased variance, as
// nn.LayerNorm); the per-lane summation order is fixed by this mapping, so layernorm_kernel and
// layernorm_pack_kernel (which both call it) agree bit for bit.  emit(j, y0..y3) stores run j.
template <typename Emit>
__device__ __forceinline__ void ln_row_vec4(const float* __restrict__ xr, int d, const float* __restrict__ gamma,
                                            const float* __restrict__ beta, double eps, Emit emit) {
  const int lane = threadIdx.x & 63;
  const int nv = d >> 2;
  float4 v[4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
    v[m] = (lane + 64 * m < nv) ? reinterpret_cast<const float4*>(xr)[lane + 64 * m] : make_float4(0.f, 0.f, 0.f, 0.f);
  double s = 0.0;
#pragma unroll
  for (int m = 0; m < 4; ++m)
    if (lane + 64 * m < nv) s = (((s + (double)v[m].x) + (double)v[m].y) + (double)v[m].z) + (double)v[m].w;
  const double mean = wave_sum(s) / (double)d;
  double q = 0.0;
#pragma unroll
  for (int m = 0; m < 4; ++m)
    if (lane + 64 * m < nv) {
      const double c0 = (double)v[m].x - mean, c1 = (double)v[m].y - mean;
      const double c2 = (double)v[m].z - mean, c3 = (double)v[m].w - mean;
      q = fma(c3, c3, fma(c2, c2, fma(c1, c1, fma(c0, c0, q))));
    }
  const double rstd = 1.0 / sqrt(wave_sum(q) / (double)d + eps);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int j = lane + 64 * m;
    if (j < nv) {
      const float4 g = gamma ? reinterpret_cast<const float4*>(gamma)[j] : make_float4(1.f, 1.f, 1.f, 1.f);
      const float4 b = beta ? reinterpret_cast<const float4*>(beta)[j] : make_float4(0.f, 0.f, 0.f, 0.f);
      emit(j, (float)((((double)v[m].x - mean) * rstd) * (double)g.x + (double)b.x),
           (float)((((double)v[m].y - mean) * rstd) * (double)g.y + (double)b.y),
           (float)((((double)v[m].z - mean) * rstd) * (double)g.z + (double)b.z),
           (float)((((double)v[m].w - mean) * rstd) * (double)g.w + (double)b.w));
    }
  }
}

template <bool VEC4>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int64_t ldx, int64_t n,
                                                        int64_t d, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, double eps,
                                                        float* __restrict__ y, int64_t ldy) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const float* xr = x + row * ldx;
  if constexpr (VEC4) {  // chosen on the INPUT side only (ln_vec4_ok); the output may be unaligned
    float* yr = y + row * ldy;
    const bool yvec = ((ldy & 3) == 0) && (((uintptr_t)y & 15) == 0);
    ln_row_vec4(xr, (int)d, gamma, beta, eps, [&](int j, float a, float b, float c, float e) {
      if (yvec) {
        reinterpret_cast<float4*>(yr)[j] = make_float4(a, b, c, e);
      } else {
        yr[4 * j] = a;
        yr[4 * j + 1] = b;
        yr[4 * j + 2] = c;
        yr[4 * j + 3] = e;
      }
    });
    return;
  }
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

// Same attention, block per batch element b with ALL heads: lane l owns elements [E l, E l + E)
// of every K / V row (E = d / 64, a head = dh / E consecutive lanes), so each key row is one
// coalesced 4*d-byte read per wave and a head's q.k is a DPP sum over its lanes; the softmax and
// the V accumulation keep mha_1q_kernel's arithmetic and order (only the q.k partial-sum order
// differs).  The per-(b, h) kernel read 80-float row pieces and reduced each key over 64 lanes
// with LDS permutes: ~2.2 TB/s on the C4 shape.
__device__ __forceinline__ float group_sum_f32(float v, int lph) {
  auto dpp = [](float x, int ctrl) -> float {
    switch (ctrl) {
      case 0: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));
      case 1: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));
      case 2: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xF, 0xF, false));
      default: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xF, 0xF, false));
    }
  };
  if (lph >= 2) v += dpp(v, 0);   // quad_perm [1,0,3,2]
  if (lph >= 4) v += dpp(v, 1);   // quad_perm [2,3,0,1]
  if (lph >= 8) v += dpp(v, 2);   // row_half_mirror
  if (lph >= 16) v += dpp(v, 3);  // row_mirror
  return v;
}

template <int E>
__global__ __launch_bounds__(256) void mha_1q_rows_kernel(const float* __restrict__ q, int64_t ldq,
                                                          const float* __restrict__ kv, int64_t ldkv, int64_t v_off,
                                                          int B, int T, int H, int dh, float* __restrict__ out,
                                                          int64_t ldo) {
  extern __shared__ float sh[];  // scores [H][T] + partial out [4][d]
  constexpr int D = 64 * E;
  float* sc = sh;
  float* po = sc + (size_t)H * T;
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lph = dh / E, head = lane / lph;
  const float scaling = 1.0f / sqrtf((float)dh);
  float qv[E];
#pragma unroll
  for (int i = 0; i < E; ++i) qv[i] = q[(int64_t)b * ldq + lane * E + i] * scaling;
  for (int t = wave; t < T; t += 4) {
    const float* kr = kv + ((int64_t)t * B + b) * ldkv + lane * E;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < E; ++i) acc = fmaf(qv[i], kr[i], acc);
    acc = group_sum_f32(acc, lph);
    if (lane % lph == 0) sc[head * T + t] = acc;
  }
  __syncthreads();
  for (int hh = wave; hh < H; hh += 4) {  // softmax over T: mha_1q_kernel's arithmetic, one wave per head
    float* s_h = sc + (size_t)hh * T;
    float m = -INFINITY;
    for (int t = lane; t < T; t += 64) m = fmaxf(m, s_h[t]);
    m = wave_max(m);
    double s = 0.0;
    for (int t = lane; t < T; t += 64) {
      const float p = expf(s_h[t] - m);
      s_h[t] = p;
      s += (double)p;
    }
    s = wave_sum(s);
    const float inv = (float)(1.0 / s);
    for (int t = lane; t < T; t += 64) s_h[t] *= inv;
  }
  __syncthreads();
  float acc[E];
#pragma unroll
  for (int i = 0; i < E; ++i) acc[i] = 0.f;
  for (int t = wave; t < T; t += 4) {
    const float p = sc[head * T + t];
    const float* vr = kv + ((int64_t)t * B + b) * ldkv + v_off + lane * E;
#pragma unroll
    for (int i = 0; i < E; ++i) acc[i] = fmaf(p, vr[i], acc[i]);
  }
#pragma unroll
  for (int i = 0; i < E; ++i) po[wave * D + lane * E + i] = acc[i];
  __syncthreads();
  for (int e = tid; e < D; e += 256)
    out[(int64_t)b * ldo + e] = (po[e] + po[D + e]) + (po[2 * D + e] + po[3 * D + e]);
}

// ---------------------------------------------------------------------------
// K9b: the Combiner's attention with its K / V in-projections ABSORBED into the query and output
// sides (combiner.py:38-40 with k = v = p_s_m.reshape(l*f, b, d), combiner.py:164-166).  Per head h,
// with n_t = (x_t - mean_t) * rstd_t the un-affined LayerNorm of key row x_t:
//   q'_h . K_t,h = n_t . (gamma (.) W_k,h^T q'_h) + (terms constant over t: softmax-invariant, dropped)
//   sum_t p_t V_t,h = W_v,h (gamma (.) z_h + beta) + b_v,h,   z_h = sum_t p_t n_t
// so the host folds W_k into the query GEMM (u_h = gamma (.) W_k,h^T (W_q,h ln(q) + b_q,h) / sqrt(dh), one
// [d] -> [H d] GEMM) and W_v / out_proj into one [H d] -> [d] GEMM after this kernel, and the 128 key rows
// of a query are never projected: 2 * 128 * d * 2d MACs per query become ~2 * H * d * d.  This kernel
// reads the key rows STRAIGHT from the conv1x1 GEMM output y ([B f npix, C]: row (bf, p), column c = the
// conv output at channel c, pixel p), whose raw reshape (combiner.py:159,164) makes key run r of block bf
// the channels [r cpr, (r + 1) cpr) x all npix pixels (cpr = d / npix): no transpose, no LayerNorm pass,
// no K / V matrix.  Kernel element order within a run: e = p * cpr + c'  (original element c' npix + p);
// the host permutes the absorbed weights to match.  One wave per query, all H heads, online softmax
// (running max / sum per head); v.mean(0) (combiner.py:40) from the same rows.  LayerNorm statistics in
// fp32 two-pass (torch's fp32 LayerNorm subclass, combiner.py:11-17).
__device__ __forceinline__ float wave_sum_f32(float v) {  // every lane gets the same bits
  v = group_sum_f32(v, 16);
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
}

template <int E, int HW, int NWV, int R>  // HW heads per wave, NWV waves per block (one query): H = HW * NWV;
// R key rows per step, their 2 + HW wave sums interleaved.  The lane's elements are handled in pairs on the packed
// fp32 pipe (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two lanes' worth of work per instruction): the kernel is
// VALU-bound (~300 instructions per key row and wave before), not load-bound
__global__ __launch_bounds__(64 * NWV, 3) void mha_absorbed_kernel(const float* __restrict__ y, int64_t ldy, int npix, int cpr,
                                                          int L, int f, int gs, const float* __restrict__ u,
                                                          int64_t ldu, float eps, float* __restrict__ z, int64_t ldz,
                                                          float* __restrict__ vmean, int64_t ldv) {
  constexpr int D = 64 * E, E2 = E / 2, H = HW;
  typedef float f2v __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // heads [wv HW, (wv + 1) HW)
  // neighbouring queries of a group read neighbouring 160-B key runs of the same conv rows (their cache lines
  // overlap): XCD-contiguous query ranges keep those lines in one L2 instead of fetching them into two or three
  const int64_t qb = xcd_linear((int)blockIdx.x, (int)gridDim.x);
  const int64_t g = qb / gs, bb = qb - g * gs;
  const int T = f * L, cpr2 = cpr >> 1;
  int off[E2];  // this lane's float2 pieces of a key run: pixel p, channel pair c2 (byte offsets < 2^31)
#pragma unroll
  for (int m = 0; m < E2; ++m) {
    const int fi = lane + 64 * m, p = fi / cpr2, c2 = fi - p * cpr2;
    off[m] = 4 * (p * (int)ldy + 2 * c2);
  }
  const int span = 4 * (int)((npix - 1) * ldy + cpr);  // a key run's byte span from its first element
  auto load_run = [&](const float* base, f2v (&v)[E2]) {  // buffer loads: the run base in SGPRs, 32-bit offsets
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, span, 0x00020000);
#pragma unroll
    for (int m = 0; m < E2; ++m) v[m] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs, off[m], 0, 0));
  };
  f2v uu[H][E2];
#pragma unroll
  for (int h = 0; h < H; ++h)
#pragma unroll
    for (int m = 0; m < E2; ++m) uu[h][m] = *(const f2v*)(u + qb * ldu + (wv * HW + h) * D + 2 * (lane + 64 * m));
  auto row_base = [&](int t) {  // (32-bit division: the int64 one carries a branch that splits the row loop)
    const unsigned Rw = (unsigned)(t * gs + (int)bb), Lu = (unsigned)L;
    const unsigned rq = Rw / Lu, rr = Rw - rq * Lu;
    const int64_t bf = g * gs * f + (int64_t)rq;
    return y + bf * npix * ldy + (int64_t)rr * cpr;
  };
  f2v acc[H][E2], vs[E2];
  float mx[H], sm[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    mx[h] = -INFINITY;
    sm[h] = 0.f;
#pragma unroll
    for (int m = 0; m < E2; ++m) acc[h][m] = f2v{0.f, 0.f};
  }
#pragma unroll
  for (int m = 0; m < E2; ++m) vs[m] = f2v{0.f, 0.f};
  // one step: R key rows from buf (LayerNorm statistics, the HW head scores, the online softmax row by row)
  auto step = [&](f2v (&x)[R][E2]) {
    float mean[R], rstd[R], dot[R][H];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      f2v s2 = {0.f, 0.f};
#pragma unroll
      for (int m = 0; m < E2; ++m) {
        s2 += x[r][m];
        vs[m] += x[r][m];
      }
      mean[r] = wave_sum_f32(s2.x + s2.y) / (float)D;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const f2v mn = {mean[r], mean[r]};
      f2v q2 = {0.f, 0.f};
      f2v a2[H];
#pragma unroll
      for (int h = 0; h < H; ++h) a2[h] = f2v{0.f, 0.f};
#pragma unroll
      for (int m = 0; m < E2; ++m) {
        x[r][m] -= mn;
        q2 = __builtin_elementwise_fma(x[r][m], x[r][m], q2);
#pragma unroll
        for (int h = 0; h < H; ++h) a2[h] = __builtin_elementwise_fma(x[r][m], uu[h][m], a2[h]);
      }
      rstd[r] = 1.0f / sqrtf(wave_sum_f32(q2.x + q2.y) / (float)D + eps);
#pragma unroll
      for (int h = 0; h < H; ++h) dot[r][h] = wave_sum_f32(a2[h].x + a2[h].y) * rstd[r];  // wave-uniform scores
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const f2v rs2 = {rstd[r], rstd[r]};
#pragma unroll
      for (int m = 0; m < E2; ++m) x[r][m] *= rs2;
#pragma unroll
      for (int h = 0; h < H; ++h) {
        // branch-free online softmax (a branch per head split the step into blocks, and the compiler then sank the
        // next rows' loads below them): k = 1 exactly when the maximum stays, so the rescale is a no-op there;
        // one exponential per head and row: with the new maximum nm = max(mx, sc), one of exp(mx - nm), exp(sc - nm)
        // is exp(0) = 1 and the other is exp(-|sc - mx|) (exact negation: the same bits as computing it directly)
        const float sc = dot[r][h];
        const bool up = sc > mx[h];
        const float e = expf(up ? mx[h] - sc : sc - mx[h]);  // 0 on the first row (mx = -inf)
        const float k = up ? e : 1.f, p = up ? 1.f : e;
        mx[h] = up ? sc : mx[h];
        sm[h] = __fadd_rn(__fmul_rn(sm[h], k), p);
        const f2v k2 = {k, k}, p2 = {p, p};
#pragma unroll
        for (int m = 0; m < E2; ++m) acc[h][m] = __builtin_elementwise_fma(p2, x[r][m], acc[h][m] * k2);
      }
    }
  };
  auto issue = [&](int t, f2v (&buf)[R][E2]) {  // rows t .. t + R - 1 (past the last row: the last row again)
#pragma unroll
    for (int r = 0; r < R; ++r) load_run(row_base(min(t + r, T - 1)), buf[r]);
    __builtin_amdgcn_sched_barrier(0);
  };
  // two named buffers in ping-pong (no register copy between a load and its use: with one prefetch buffer copied
  // into the working rows, the compiler placed the copy -- and a wait for the prefetch -- at the loop's back edge,
  // so every row waited out a full memory round trip)
  f2v ba[R][E2], bb2[R][E2];
  issue(0, ba);
  int t0 = 0;
  for (; t0 + 2 * R <= T; t0 += 2 * R) {
    issue(t0 + R, bb2);
    step(ba);
    issue(t0 + 2 * R, ba);
    step(bb2);
  }
  if (t0 < T) step(ba);  // (T an odd multiple of R)
#pragma unroll
  for (int h = 0; h < H; ++h) {
    const float inv = 1.0f / sm[h];
    const f2v i2 = {inv, inv};
#pragma unroll
    for (int m = 0; m < E2; ++m) *(f2v*)(z + qb * ldz + (wv * HW + h) * D + 2 * (lane + 64 * m)) = acc[h][m] * i2;
  }
  if (wv != 0) return;  // v.mean(0): wave 0's sums
  const float invT = 1.0f / (float)T;
#pragma unroll
  for (int m = 0; m < E2; ++m) {
    const int fi = lane + 64 * m, p = fi / cpr2, c0 = 2 * (fi - p * cpr2);
    vmean[qb * ldv + (int64_t)c0 * npix + p] = vs[m].x * invT;
    vmean[qb * ldv + (int64_t)(c0 + 1) * npix + p] = vs[m].y * invT;
  }
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


// ---------------------------------------------------------------------------
// block transposes: block b of x is [R][C] row-major; out row (b, c) = column c of block b.
// One workgroup per block, staged through LDS with a padded row (C + 1) so the column reads
// are conflict-free; OUT_PACK writes the split-bf16 planes of a raw GEMM operand
// (hi = bf16(v), lo = bf16(v - hi): pack_rows_kernel's CMVE_PACK_RAW split), else fp32.
// ---------------------------------------------------------------------------
constexpr int TB_MAX = 12288;  // R * C floats staged per block (48 KiB + padding)

// kv remap (fp32 out only, kv_d > 0): the transposed blocks form a flat array whose consecutive
// kv_d-float runs u are the raw p_s_m.reshape(G, T, gs, d) rows (g, t, bb) = (u / (T gs),
// (u / gs) % T, u % gs); run u is written to row t*kvB + g*gs + bb -- the key/value order of
// combiner.py:164-165 for G consecutive batches of gs rows (G = 1: the plain reshape).
// V = 4: float4 block loads (C % 4 == 0) and four consecutive outputs of one row per thread
// (row width % 4 == 0; a kv run then holds all four) -- one index computation per four elements and
// 16-byte fp32 / 8-byte bf16 stores; V = 1 is the scalar form for the other shapes.
template <bool OUT_PACK, int V>
__global__ __launch_bounds__(256) void tblocks_kernel(const float* __restrict__ x, int64_t nb, int R, int C,
                                                      float* __restrict__ y, uint16_t* __restrict__ hi,
                                                      uint16_t* __restrict__ lo, int64_t d_pad, int kv_d = 0,
                                                      int kv_T = 1, int kv_gs = 1, int kv_B = 1) {
  extern __shared__ float tb[];  // [R][C + 1]
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const int W = R * C;
  const int S = C + 1;
  if (b < nb) {
    const float* xb = x + b * (int64_t)W;
    if constexpr (V == 4) {
      for (int e4 = tid; e4 < (W >> 2); e4 += 256) {
        const float4 v = reinterpret_cast<const float4*>(xb)[e4];
        const int r = (e4 << 2) / C, c = (e4 << 2) - r * C;
        float* t = tb + r * S + c;
        t[0] = v.x;
        t[1] = v.y;
        t[2] = v.z;
        t[3] = v.w;
      }
    } else {
      for (int e = tid; e < W; e += 256) tb[(e / C) * S + (e % C)] = xb[e];
    }
    __syncthreads();
  }
  const int ow = OUT_PACK ? (int)d_pad : R;  // output row width
  const int owv = ow / V;
  for (int ev = tid; ev < C * owv; ev += 256) {
    const int c = ev / owv, k = (ev - c * owv) * V;
    float v[V];
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = (b < nb && k + j < R) ? tb[(k + j) * S + c] : 0.f;
    int64_t o = (b * C + c) * (int64_t)ow + k;
    if constexpr (OUT_PACK) {
      uint16_t hh[V], ll[V];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        hh[j] = f2bf(v[j]);
        ll[j] = f2bf(v[j] - bf2f(hh[j]));
      }
      if constexpr (V == 4) {
        reinterpret_cast<uint2*>(hi + o)[0] = make_uint2(hh[0] | ((uint32_t)hh[1] << 16), hh[2] | ((uint32_t)hh[3] << 16));
        reinterpret_cast<uint2*>(lo + o)[0] = make_uint2(ll[0] | ((uint32_t)ll[1] << 16), ll[2] | ((uint32_t)ll[3] << 16));
      } else {
        hi[o] = hh[0];
        lo[o] = ll[0];
      }
    } else {
      if (kv_d > 0) {  // 32-bit index math (the host checks nb * R * C < 2^32)
        const uint32_t ou = (uint32_t)o, u = ou / (uint32_t)kv_d, w = ou - u * (uint32_t)kv_d;
        const uint32_t tg = (uint32_t)kv_T * (uint32_t)kv_gs, g = u / tg, rem = u - g * tg;
        const uint32_t t = rem / (uint32_t)kv_gs, bb = rem - t * (uint32_t)kv_gs;
        o = ((int64_t)t * kv_B + (int64_t)g * kv_gs + bb) * kv_d + w;
      }
      if constexpr (V == 4)
        reinterpret_cast<float4*>(y + o)[0] = make_float4(v[0], v[1], v[2], v[3]);
      else
        y[o] = v[0];
    }
  }
}

// LayerNorm of rows of x (the register-row path of layernorm_kernel, same arithmetic) written as
// the split-bf16 planes of a raw GEMM operand; rows [n, n_pad) and columns [d, d_pad) are zero.
template <bool VEC4>
__global__ __launch_bounds__(256) void layernorm_pack_kernel(const float* __restrict__ x, int64_t ldx, int64_t n,
                                                             int64_t d, int64_t n_pad, int64_t d_pad,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, double eps,
                                                             uint16_t* __restrict__ hi, uint16_t* __restrict__ lo) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n_pad) return;
  uint16_t* hr = hi + row * d_pad;
  uint16_t* lr = lo + row * d_pad;
  if (row >= n) {
    for (int64_t k = lane; k < d_pad; k += 64) hr[k] = lr[k] = 0;
    return;
  }
  const float* xr = x + row * ldx;
  if constexpr (VEC4) {  // chosen on the INPUT side only (ln_vec4_ok); 8-byte stores when the planes allow
    const bool ovec = ((d_pad & 3) == 0) && (((uintptr_t)hi & 7) == 0) && (((uintptr_t)lo & 7) == 0);
    ln_row_vec4(xr, (int)d, gamma, beta, eps, [&](int j, float a, float b, float c, float e) {
      const uint16_t h0 = f2bf(a), h1 = f2bf(b), h2 = f2bf(c), h3 = f2bf(e);
      const uint16_t l0 = f2bf(a - bf2f(h0)), l1 = f2bf(b - bf2f(h1)), l2 = f2bf(c - bf2f(h2)),
                     l3 = f2bf(e - bf2f(h3));
      if (ovec) {
        reinterpret_cast<uint2*>(hr)[j] = make_uint2(h0 | ((uint32_t)h1 << 16), h2 | ((uint32_t)h3 << 16));
        reinterpret_cast<uint2*>(lr)[j] = make_uint2(l0 | ((uint32_t)l1 << 16), l2 | ((uint32_t)l3 << 16));
      } else {
        hr[4 * j] = h0; hr[4 * j + 1] = h1; hr[4 * j + 2] = h2; hr[4 * j + 3] = h3;
        lr[4 * j] = l0; lr[4 * j + 1] = l1; lr[4 * j + 2] = l2; lr[4 * j + 3] = l3;
      }
    });
    for (int64_t k = d + lane; k < d_pad; k += 64) hr[k] = lr[k] = 0;
    return;
  }
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
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int64_t k = lane + 64 * m;
    if (k < d) {
      const double c = ((double)v[m] - mean) * rstd;
      const float y = (float)(c * (double)(gamma ? gamma[k] : 1.f) + (double)(beta ? beta[k] : 0.f));
      const uint16_t h = f2bf(y);
      hr[k] = h;
      lr[k] = f2bf(y - bf2f(h));
    }
  }
  for (int64_t k = d + lane; k < d_pad; k += 64) hr[k] = lr[k] = 0;
}

}  // namespace cmve

using namespace cmve;

static bool a16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// tblocks_kernel<., 4>: float4 block loads (C % 4 == 0, 16-byte x) and output rows of ow % 4 == 0
static bool tb_vec4(const float* x, int64_t C, int64_t ow) { return C % 4 == 0 && ow % 4 == 0 && a16(x); }

// float4 rows for ln_row_vec4: d <= 1024 and every row / gamma / beta 16-byte aligned
static bool ln_vec4_ok(const float* x, int64_t ldx, int64_t d, const float* gamma, const float* beta) {
  return d <= 1024 && d % 4 == 0 && ldx % 4 == 0 && a16(x) && (!gamma || a16(gamma)) && (!beta || a16(beta));
}

extern "C" int cmve_layernorm(cmve_handle_t h, const float* x, int64_t ldx, int64_t n, int64_t d, const float* gamma,
                              const float* beta, double eps, float* y, int64_t ldy) {
  CMVE_REQUIRE(h && x && y, "cmve_layernorm: NULL argument");
  CMVE_REQUIRE(n >= 0 && d > 0 && ldx >= d && ldy >= d, "cmve_layernorm: bad shape");
  if (n == 0) return CMVE_OK;
  // path chosen on the input side only, so cmve_layernorm and cmve_layernorm_pack sum in the same order
  if (ln_vec4_ok(x, ldx, d, gamma, beta))
    hipLaunchKernelGGL(layernorm_kernel<true>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, h->stream, x, ldx, n, d,
                       gamma, beta, eps, y, ldy);
  else
    hipLaunchKernelGGL(layernorm_kernel<false>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, h->stream, x, ldx, n, d,
                       gamma, beta, eps, y, ldy);
  return check_launch("layernorm");
}

extern "C" int cmve_mha_1q(cmve_handle_t h, const float* q, int64_t ldq, const float* kv, int64_t ldkv, int64_t v_off,
                           int32_t B, int32_t T, int32_t H, int32_t dh, float* out, int64_t ldo) {
  CMVE_REQUIRE(h && q && kv && out, "cmve_mha_1q: NULL argument");
  CMVE_REQUIRE(B > 0 && T > 0 && H > 0 && dh > 0 && ldq >= (int64_t)H * dh && ldo >= (int64_t)H * dh,
               "cmve_mha_1q: bad shape");
  const int64_t d = (int64_t)H * dh;
  const int E = (int)(d / 64);
  const int lph = (d % 64 == 0 && E > 0 && dh % E == 0) ? dh / E : 0;
  const size_t lds_rows = sizeof(float) * ((size_t)H * T + 4 * (size_t)d);
  if ((E == 10 || E == 8 || E == 16 || E == 4) && (lph == 1 || lph == 2 || lph == 4 || lph == 8 || lph == 16) &&
      lds_rows <= 64 * 1024) {  // all heads per block (Combiner: d 640 = 8 x 80, E 10)
#define MR(EE)                                                                                                       hipLaunchKernelGGL(mha_1q_rows_kernel<EE>, dim3((unsigned)B), dim3(256), lds_rows, h->stream, q, ldq, kv, ldkv,                      v_off, B, T, H, dh, out, ldo)
    if (E == 10) MR(10);
    else if (E == 8) MR(8);
    else if (E == 16) MR(16);
    else MR(4);
#undef MR
    return check_launch("mha_1q_rows");
  }
  const size_t lds = sizeof(float) * ((size_t)T + dh + 4 * (size_t)dh);
  CMVE_REQUIRE(lds <= 64 * 1024, "cmve_mha_1q: T/dh too large for one block");
  hipLaunchKernelGGL(mha_1q_kernel, dim3((unsigned)B, (unsigned)H), dim3(256), lds, h->stream, q, ldq, kv, ldkv, v_off,
                     B, T, H, dh, out, ldo);
  return check_launch("mha_1q");
}

extern "C" int cmve_mha_absorbed(cmve_handle_t h, const float* y, int64_t ldy, int64_t C, int64_t npix, int64_t f,
                                 int64_t gs, int64_t B, int32_t H, int64_t d, const float* u, int64_t ldu, double eps,
                                 float* z, int64_t ldz, float* vmean, int64_t ldv) {
  CMVE_REQUIRE(h && y && u && z && vmean, "cmve_mha_absorbed: NULL argument");
  CMVE_REQUIRE(B >= 0 && f > 0 && gs > 0 && B % gs == 0 && npix > 0 && C > 0 && d > 0 && H > 0,
               "cmve_mha_absorbed: bad shape (B a multiple of gs)");
  CMVE_REQUIRE(d % npix == 0 && (d / npix) % 2 == 0 && C % (d / npix) == 0,
               "cmve_mha_absorbed: d / npix channels per key run, even, dividing C");
  CMVE_REQUIRE(ldy >= C && ldu >= H * d && ldz >= H * d && ldv >= d && ldy % 2 == 0 && ldu % 2 == 0 && ldz % 2 == 0 &&
                   ((uintptr_t)y & 7) == 0 && ((uintptr_t)u & 7) == 0 && ((uintptr_t)z & 7) == 0,
               "cmve_mha_absorbed: strides / 8-byte alignment");
  if (B == 0) return CMVE_OK;
  const int cpr = (int)(d / npix), L = (int)(C / cpr);
  CMVE_REQUIRE(4 * npix * ldy < ((int64_t)1 << 31), "cmve_mha_absorbed: a key block's span exceeds 2 GiB");
#ifndef CMVE_MHA_ROWS
#define CMVE_MHA_ROWS 1  // key rows per step (1, 2 or 4; a study build's -D)
#endif
#ifndef CMVE_MHA_HPW
#define CMVE_MHA_HPW 4  // heads per wave (4: two waves per query, 2: four; a study build's -D)
#endif
  constexpr int rows = (CMVE_MHA_ROWS == 2 || CMVE_MHA_ROWS == 4) ? CMVE_MHA_ROWS : 1;
  // (round 4, tools/ab_mha.sh at C4 size: 4 heads x 1 row 36.4 ms per combine_batches pass, 4 x 2 36.7, 2 x 1 37.9,
  // 2 x 2 37.8, 2 x 4 38.5 -- four waves read every key row twice as often, and more rows per step only add
  // registers: the kernel is not waiting on its loads)
  constexpr int hpw = CMVE_MHA_HPW == 2 ? 2 : 4;
  const int T = (int)(f * L), R = (T % rows == 0) ? rows : ((T % 2 == 0) ? 2 : 1);
#define CMVE_MHA_LAUNCH(E_, HW_, R_)                                                                                 \
  hipLaunchKernelGGL((mha_absorbed_kernel<E_, HW_, 8 / HW_, R_>), dim3((unsigned)B), dim3(64 * (8 / HW_)), 0,         \
                     h->stream, y, ldy, (int)npix, cpr, L, (int)f, (int)gs, u, ldu, (float)eps, z, ldz, vmean, ldv)
#define CMVE_MHA_R(E_, HW_)             \
  if (R == 4) CMVE_MHA_LAUNCH(E_, HW_, 4); \
  else if (R == 2) CMVE_MHA_LAUNCH(E_, HW_, 2); \
  else CMVE_MHA_LAUNCH(E_, HW_, 1)
  if ((d == 640 || d == 512) && H == 8) {  // the Combiner: d 640 = 64 lanes x 10, 8 heads
    if (d == 640) {
      if (hpw == 4) { CMVE_MHA_R(10, 4); }
      else { CMVE_MHA_R(10, 2); }
    } else {
      if (hpw == 4) { CMVE_MHA_R(8, 4); }
      else { CMVE_MHA_R(8, 2); }
    }
#undef CMVE_MHA_R
#undef CMVE_MHA_LAUNCH
    return check_launch("mha_absorbed");
  }
  set_error("cmve_mha_absorbed: instantiated for (d, H) = (640, 8), (512, 8)");
  return CMVE_E_UNSUPPORTED;
}

extern "C" int cmve_fuse_combine(cmve_handle_t h, const float* y, const float* ds, const float* text, const float* ref,
                                 const float* based, int64_t n, int64_t d, double eps, float* out) {
  CMVE_REQUIRE(h && y && ds && text && ref && based && out, "cmve_fuse_combine: NULL argument");
  if (n == 0) return CMVE_OK;
  hipLaunchKernelGGL(fuse_combine_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, h->stream, y, ds, text, ref,
                     based, n, d, eps, out);
  return check_launch("fuse_combine");
}


// a raw (CMVE_PACK_RAW) GEMM operand written by a fused kernel: no score bound (err_max = +inf)
static int raw_operand_ready(cmve_handle_t h, cmve_rows_t* r) {
  r->flags |= CMVE_PACK_RAW;
  if (r->err_max) CMVE_HIP(hipMemsetD32Async((hipDeviceptr_t)r->err_max, 0x7f800000u, 3, h->stream));
  return CMVE_OK;
}

extern "C" int cmve_transpose_blocks(cmve_handle_t h, const float* x, int64_t nb, int64_t R, int64_t C, float* y) {
  CMVE_REQUIRE(h && x && y, "cmve_transpose_blocks: NULL argument");
  CMVE_REQUIRE(nb >= 0 && R > 0 && C > 0 && R * C <= TB_MAX && R * (C + 1) * 4 <= 65536,
               "cmve_transpose_blocks: bad block shape");
  if (nb == 0) return CMVE_OK;
  const size_t lds = sizeof(float) * (size_t)R * (size_t)(C + 1);
  if (tb_vec4(x, C, R) && a16(y))
    hipLaunchKernelGGL((tblocks_kernel<false, 4>), dim3((unsigned)nb), dim3(256), lds, h->stream, x, nb, (int)R,
                       (int)C, y, nullptr, nullptr, (int64_t)0);
  else
    hipLaunchKernelGGL((tblocks_kernel<false, 1>), dim3((unsigned)nb), dim3(256), lds, h->stream, x, nb, (int)R,
                       (int)C, y, nullptr, nullptr, (int64_t)0);
  return check_launch("transpose_blocks");
}

extern "C" int cmve_transpose_blocks_kv(cmve_handle_t h, const float* x, int64_t nb, int64_t R, int64_t C, int64_t d,
                                        int64_t T, int64_t gs, int64_t B, float* y) {
  CMVE_REQUIRE(h && x && y, "cmve_transpose_blocks_kv: NULL argument");
  CMVE_REQUIRE(nb >= 0 && R > 0 && C > 0 && R * C <= TB_MAX && R * (C + 1) * 4 <= 65536,
               "cmve_transpose_blocks_kv: bad block shape");
  CMVE_REQUIRE(d > 0 && T > 0 && gs > 0 && B % gs == 0 && (nb * R * C) == B * T * d,
               "cmve_transpose_blocks_kv: nb*R*C must equal B*T*d with gs | B");
  CMVE_REQUIRE(nb * R * C < (1ll << 32), "cmve_transpose_blocks_kv: more than 2^32 elements (split the batch)");
  if (nb == 0) return CMVE_OK;
  const size_t lds = sizeof(float) * (size_t)R * (size_t)(C + 1);
  if (tb_vec4(x, C, R) && d % 4 == 0 && a16(y))
    hipLaunchKernelGGL((tblocks_kernel<false, 4>), dim3((unsigned)nb), dim3(256), lds, h->stream, x, nb, (int)R,
                       (int)C, y, nullptr, nullptr, (int64_t)0, (int)d, (int)T, (int)gs, (int)B);
  else
    hipLaunchKernelGGL((tblocks_kernel<false, 1>), dim3((unsigned)nb), dim3(256), lds, h->stream, x, nb, (int)R,
                       (int)C, y, nullptr, nullptr, (int64_t)0, (int)d, (int)T, (int)gs, (int)B);
  return check_launch("transpose_blocks_kv");
}

extern "C" int cmve_pack_tblocks(cmve_handle_t h, const float* x, int64_t nb, int64_t R, int64_t C, cmve_rows_t* out) {
  CMVE_REQUIRE(h && x && out && out->hi && out->lo, "cmve_pack_tblocks: NULL argument");
  CMVE_REQUIRE(nb >= 0 && R > 0 && C > 0 && R * C <= TB_MAX && R * (C + 1) * 4 <= 65536,
               "cmve_pack_tblocks: bad block shape");
  CMVE_REQUIRE(out->n == nb * C && out->d == R && out->d_pad >= R && out->n_pad >= out->n && out->n_pad % C == 0,
               "cmve_pack_tblocks: out must describe nb*C rows of R (n_pad a multiple of C)");
  const size_t lds = sizeof(float) * (size_t)R * (size_t)(C + 1);
  const int64_t grid = out->n_pad / C;  // blocks past nb write the zero padding rows
  if (grid) {
    if (tb_vec4(x, C, out->d_pad) && ((uintptr_t)out->hi & 7) == 0 && ((uintptr_t)out->lo & 7) == 0)
      hipLaunchKernelGGL((tblocks_kernel<true, 4>), dim3((unsigned)grid), dim3(256), lds, h->stream, x, nb, (int)R,
                         (int)C, nullptr, out->hi, out->lo, out->d_pad);
    else
      hipLaunchKernelGGL((tblocks_kernel<true, 1>), dim3((unsigned)grid), dim3(256), lds, h->stream, x, nb, (int)R,
                         (int)C, nullptr, out->hi, out->lo, out->d_pad);
    int st = check_launch("pack_tblocks");
    if (st) return st;
  }
  return raw_operand_ready(h, out);
}

extern "C" int cmve_layernorm_pack(cmve_handle_t h, const float* x, int64_t ldx, int64_t n, int64_t d,
                                   const float* gamma, const float* beta, double eps, cmve_rows_t* out) {
  CMVE_REQUIRE(h && x && out && out->hi && out->lo, "cmve_layernorm_pack: NULL argument");
  CMVE_REQUIRE(n >= 0 && d > 0 && d <= 1024 && ldx >= d, "cmve_layernorm_pack: bad shape (d <= 1024)");
  CMVE_REQUIRE(out->n == n && out->d == d && out->d_pad >= d && out->n_pad >= n, "cmve_layernorm_pack: bad out");
  if (out->n_pad) {
    if (ln_vec4_ok(x, ldx, d, gamma, beta))  // input side only (see cmve_layernorm)
      hipLaunchKernelGGL(layernorm_pack_kernel<true>, dim3((unsigned)((out->n_pad + 3) / 4)), dim3(256), 0, h->stream,
                         x, ldx, n, d, out->n_pad, out->d_pad, gamma, beta, eps, out->hi, out->lo);
    else
      hipLaunchKernelGGL(layernorm_pack_kernel<false>, dim3((unsigned)((out->n_pad + 3) / 4)), dim3(256), 0,
                         h->stream, x, ldx, n, d, out->n_pad, out->d_pad, gamma, beta, eps, out->hi, out->lo);
    int st = check_launch("layernorm_pack");
    if (st) return st;
  }
  return raw_operand_ready(h, out);
}
