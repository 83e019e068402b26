// K4: N_q x N_g cosine-similarity GEMM on bf16 MFMA (gfx950), with fused epilogues.
//
//   EPI_STORE : out[i,j] = alpha * s_ij + beta            (cal_error / cal_simi / logits)
//   EPI_RANK  : per-row and per-column "score > threshold" counts + undecided-pair list
//               (the GT rank of LINAS-engine/util/metrics.py:137-147 without the matrix)
//
// Geometry: 256 threads = 4 waves (2 x 2), block tile 128 (q rows) x 128 (g rows),
// K step 64, each wave owns 64 x 64 = 4 x 4 tiles of v_mfma_f32_16x16x32_bf16.
// Staging: global_load_lds_dwordx4 (16 B / lane, 1 KiB per wave-instruction) into a
// lane-linear LDS image, 2 stages; bank conflicts removed by an XOR swizzle applied
// to the GLOBAL source chunk (chunk ^ (row & 7)) and the matching ds_read_b128 address.
// Grid: XCD-aware -- each XCD gets a contiguous range of the logical tile order and the
// logical order walks 8 gallery tiles x all query tiles, so the 64 co-resident blocks of
// an XCD share 8 G tiles and 8 Q tiles in its 4 MiB L2.
#include "cmve_internal.h"

namespace cmve {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int PLANE_BYTES = BM * BK * 2;  // 16 KiB
constexpr int EPI_STORE = 0, EPI_RANK = 1, EPI_LINEAR = 2;
constexpr int CAND_LDS = 1024;  // per-block undecided-pair buffer (one global atomic per block)

struct SimArgs {
  const uint16_t* qhi;
  const uint16_t* qlo;
  const uint16_t* ghi;
  const uint16_t* glo;
  int64_t ldk;  // d_pad
  int nq, ng;
  int nblk_m, nblk_n;
  int nk;
  // linear epilogue: v = acc + bias; relu; + resid; v * bn_scale + bn_shift
  const float* bias;
  const float* bn_scale;
  const float* bn_shift;
  const float* resid;
  int64_t ldr;
  int relu;
  // store
  void* out;
  int64_t ldo;
  float alpha, beta;
  int out_f64;
  // rank
  const float* row_hi;
  const float* row_lo;
  const float* col_hi;
  const float* col_lo;
  int* row_cnt;
  int* col_cnt;
  unsigned long long* cand;
  long long cand_cap;
  unsigned long long* cand_count;
};

// bijective XCD remap + grouped (GN gallery tiles x all query tiles) logical order
__device__ __forceinline__ void tile_of_block(int bid, int nblk_m, int nblk_n, int& bm, int& bn) {
  const int total = nblk_m * nblk_n;
  const int xcd = bid & 7, local = bid >> 3;
  const int q = total >> 3, r = total & 7;
  const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
  constexpr int GN = 8;
  const int group = L / (GN * nblk_m);
  const int within = L - group * (GN * nblk_m);
  const int gn = min(GN, nblk_n - group * GN);
  bm = within / gn;
  bn = group * GN + (within - bm * gn);
}

// issue this wave's share (4 x 1 KiB) of one 128 x 64 bf16 plane
__device__ __forceinline__ void stage_plane(const uint16_t* __restrict__ src, int64_t ldk, int row0, int k0,
                                            char* lds_plane, int wave, int lane) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int r = (wave * 4 + it) * 8 + (lane >> 3);
    const int c = lane & 7;
    const int gc = c ^ (r & 7);
    const uint16_t* g = src + (int64_t)(row0 + r) * ldk + k0 + gc * 8;
    __builtin_amdgcn_global_load_lds((const void*)g, (lds_void_t*)(lds_plane + (wave * 4 + it) * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ s16x8_t read_frag(const char* plane, int row, int chunk) {
  // row & 7 == lane & 7 for every fragment row this kernel reads
  return *(const s16x8_t*)(plane + row * 128 + ((chunk ^ (row & 7)) << 4));
}

template <int MODE>
__device__ __forceinline__ f32x4_t mfma(s16x8_t a, s16x8_t b, f32x4_t c) {
  if constexpr (MODE == CMVE_SIM_F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                  0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                   c, 0, 0, 0);
}

template <int MODE, int EPI>
__global__ __launch_bounds__(256, 2) void sim_kernel(SimArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NPLANE = (MODE == CMVE_SIM_BF16X3) ? 4 : 2;
  constexpr int STAGE_BYTES = NPLANE * PLANE_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  int bm, bn;
  tile_of_block(blockIdx.x, a.nblk_m, a.nblk_n, bm, bn);
  const int m0 = bm * BM, n0 = bn * BN;

  int* lds_rc = (int*)(smem + 2 * STAGE_BYTES);
  int* lds_cc = lds_rc + BM;
  unsigned long long* lds_cand = (unsigned long long*)(lds_cc + BN);
  unsigned* lds_ncand = (unsigned*)(lds_cand + CAND_LDS);
  if (EPI == EPI_RANK) {
    lds_rc[tid] = 0;  // 256 ints: 128 row + 128 col counters
    if (tid == 0) *lds_ncand = 0u;
  }

  auto stage = [&](int t, int s) {
    char* base = smem + s * STAGE_BYTES;
    const int k0 = t * BK;
    stage_plane(a.qhi, a.ldk, m0, k0, base, wave, lane);
    stage_plane(a.ghi, a.ldk, n0, k0, base + PLANE_BYTES, wave, lane);
    if (MODE == CMVE_SIM_BF16X3) {
      stage_plane(a.qlo, a.ldk, m0, k0, base + 2 * PLANE_BYTES, wave, lane);
      stage_plane(a.glo, a.ldk, n0, k0, base + 3 * PLANE_BYTES, wave, lane);
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int frow = lane & 15;
  for (int t = 0; t < a.nk; ++t) {
    if (t + 1 < a.nk) stage(t + 1, (t + 1) & 1);
    const char* base = smem + (t & 1) * STAGE_BYTES;
    const char* pA = base;
    const char* pB = base + PLANE_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = ks * 4 + (lane >> 4);
      s16x8_t fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = read_frag(pA, wr * 64 + i * 16 + frow, chunk);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = read_frag(pB, wc * 64 + j * 16 + frow, chunk);
      if (MODE == CMVE_SIM_BF16X3) {
        const char* pAl = base + 2 * PLANE_BYTES;
        const char* pBl = base + 3 * PLANE_BYTES;
        s16x8_t la[4], lb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) la[i] = read_frag(pAl, wr * 64 + i * 16 + frow, chunk);
#pragma unroll
        for (int j = 0; j < 4; ++j) lb[j] = read_frag(pBl, wc * 64 + j * 16 + frow, chunk);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[i][j] = mfma<MODE>(la[i], fb[j], acc[i][j]);
            acc[i][j] = mfma<MODE>(fa[i], lb[j], acc[i][j]);
          }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = mfma<MODE>(fa[i], fb[j], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---------------- epilogues ----------------
  // accumulator element (i, j, r): row = m0 + wr*64 + i*16 + (lane>>4)*4 + r, col = n0 + wc*64 + j*16 + (lane&15)
  const int rbase = m0 + wr * 64 + (lane >> 4) * 4;
  const int cbase = n0 + wc * 64 + (lane & 15);

  if constexpr (EPI == EPI_LINEAR) {
    float bj[4], sj[4], hj[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = cbase + j * 16;
      const bool ok = col < a.ng;
      bj[j] = (a.bias && ok) ? a.bias[col] : 0.f;
      sj[j] = (a.bn_scale && ok) ? a.bn_scale[col] : 1.f;
      hj[j] = (a.bn_shift && ok) ? a.bn_shift[col] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase + i * 16 + r;
        if (row >= a.nq) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = cbase + j * 16;
          if (col >= a.ng) continue;
          float v = acc[i][j][r] + bj[j];
          if (a.relu == 1) v = fmaxf(v, 0.f);                                   // ReLU
          else if (a.relu == 2) v = v / (1.f + expf(-1.702f * v));            // QuickGELU x*sigmoid(1.702x)
          else if (a.relu == 3) v = 1.f / (1.f + expf(-v));                   // Sigmoid
          if (a.resid) v = a.resid[(int64_t)row * a.ldr + col] + v;
          if (a.bn_scale) v = v * sj[j] + hj[j];
          ((float*)a.out)[(int64_t)row * a.ldo + col] = v;
        }
      }
  } else if constexpr (EPI == EPI_STORE) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase + i * 16 + r;
        if (row >= a.nq) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = cbase + j * 16;
          if (col >= a.ng) continue;
          const float v = a.alpha * acc[i][j][r] + a.beta;
          if (a.out_f64)
            ((double*)a.out)[(int64_t)row * a.ldo + col] = (double)v;
          else
            ((float*)a.out)[(int64_t)row * a.ldo + col] = v;
        }
      }
  } else {
    // thresholds (+inf disables a direction / a padded row or column)
    f32x4_t rhi[4], rlo[4];
    float chi[4], clo[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (a.row_hi) {
        rhi[i] = *(const f32x4_t*)(a.row_hi + rbase + i * 16);
        rlo[i] = *(const f32x4_t*)(a.row_lo + rbase + i * 16);
      } else {
        rhi[i] = f32x4_t{INFINITY, INFINITY, INFINITY, INFINITY};
        rlo[i] = rhi[i];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      chi[j] = a.col_hi ? a.col_hi[cbase + j * 16] : INFINITY;
      clo[j] = a.col_lo ? a.col_lo[cbase + j * 16] : INFINITY;
    }
    const bool padded = (m0 + BM > a.nq) || (n0 + BN > a.ng);
    uint32_t rc_pack[4] = {0u, 0u, 0u, 0u};  // byte r of rc_pack[i]: count for row (i, r)
    uint32_t cc_pack = 0u;                    // byte j: count for column j
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float s = acc[i][j][r];
          const int row = rbase + i * 16 + r;
          const int col = cbase + j * 16;
          if (padded && (row >= a.nq || col >= a.ng)) s = -INFINITY;
          const bool br = s > rhi[i][r];
          const bool bc = s > chi[j];
          rc_pack[i] += (uint32_t)br << (8 * r);
          cc_pack += (uint32_t)bc << (8 * j);
          const uint32_t flags = (uint32_t)((s >= rlo[i][r]) & !br) | ((uint32_t)((s >= clo[j]) & !bc) << 1);
          if (flags) {
            const unsigned long long packed =
                (unsigned long long)row | ((unsigned long long)col << 31) | ((unsigned long long)flags << 62);
            const unsigned p = atomicAdd(lds_ncand, 1u);
            if (p < (unsigned)CAND_LDS) {
              lds_cand[p] = packed;
            } else {  // block buffer full: straight to the global list
              const unsigned long long slot = atomicAdd(a.cand_count, 1ull);
              if ((long long)slot < a.cand_cap) a.cand[slot] = packed;
            }
          }
        }
    // rows: reduce over the 16 lanes that share (lane >> 4); bytes stay <= 64
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t v = rc_pack[i];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      rc_pack[i] = v;
    }
    cc_pack += __shfl_xor(cc_pack, 16, 64);
    cc_pack += __shfl_xor(cc_pack, 32, 64);
    if ((lane & 15) == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t c = (rc_pack[i] >> (8 * r)) & 0xffu;
          if (c) atomicAdd(&lds_rc[wr * 64 + i * 16 + (lane >> 4) * 4 + r], (int)c);
        }
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t c = (cc_pack >> (8 * j)) & 0xffu;
        if (c) atomicAdd(&lds_cc[wc * 64 + j * 16 + lane], (int)c);
      }
    }
    __syncthreads();
    // flush the block's undecided pairs with ONE global atomic
    __shared__ unsigned long long cand_base;
    const unsigned nlds = min(*lds_ncand, (unsigned)CAND_LDS);
    if (tid == 0 && nlds) cand_base = atomicAdd(a.cand_count, (unsigned long long)nlds);
    __syncthreads();
    for (unsigned t = tid; t < nlds; t += 256) {
      const unsigned long long slot = cand_base + t;
      if ((long long)slot < a.cand_cap) a.cand[slot] = lds_cand[t];
    }
    if (tid < BM) {
      const int c = lds_rc[tid];
      if (c && a.row_cnt && m0 + tid < a.nq) atomicAdd(&a.row_cnt[m0 + tid], c);
    } else {
      const int c = lds_cc[tid - BM];
      if (c && a.col_cnt && n0 + tid - BM < a.ng) atomicAdd(&a.col_cnt[n0 + tid - BM], c);
    }
  }
}

template <int MODE, int EPI>
static int launch_sim(const SimArgs& a, hipStream_t stream) {
  constexpr int NPLANE = (MODE == CMVE_SIM_BF16X3) ? 4 : 2;
  const size_t lds = 2 * (size_t)NPLANE * PLANE_BYTES +
                     (EPI == EPI_RANK ? 2 * 128 * sizeof(int) + CAND_LDS * sizeof(unsigned long long) + 16 : 0);
  static bool attr_done = false;
  if (!attr_done) {
    CMVE_HIP(hipFuncSetAttribute((const void*)sim_kernel<MODE, EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lds));
    attr_done = true;
  }
  const unsigned nblocks = (unsigned)a.nblk_m * (unsigned)a.nblk_n;
  hipLaunchKernelGGL((sim_kernel<MODE, EPI>), dim3(nblocks), dim3(256), lds, stream, a);
  return check_launch("sim_kernel");
}

static int validate_pair(const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, const char* fn) {
  CMVE_REQUIRE(q && g, "%s: NULL rows", fn);
  CMVE_REQUIRE(q->d == g->d && q->d_pad == g->d_pad, "%s: dimension mismatch (%lld vs %lld)", fn, (long long)q->d,
               (long long)g->d);
  CMVE_REQUIRE(q->n_pad % BM == 0 && g->n_pad % BN == 0 && q->d_pad % BK == 0, "%s: sets not packed/padded", fn);
  CMVE_REQUIRE(q->n <= q->n_pad && g->n <= g->n_pad, "%s: n > n_pad", fn);
  CMVE_REQUIRE(q->n < (1ll << 31) && g->n < (1ll << 31), "%s: set too large for int32 indices", fn);
  CMVE_REQUIRE(mode == CMVE_SIM_BF16 || mode == CMVE_SIM_BF16X3 || mode == CMVE_SIM_F16, "%s: unknown mode %d", fn,
               mode);
  CMVE_REQUIRE(q->hi && g->hi, "%s: hi plane missing", fn);
  if (mode == CMVE_SIM_BF16X3) CMVE_REQUIRE(q->lo && g->lo, "%s: BF16X3 needs lo planes", fn);
  if (mode == CMVE_SIM_F16) CMVE_REQUIRE(q->h16 && g->h16, "%s: F16 needs h16 planes", fn);
  return CMVE_OK;
}

static SimArgs make_args(const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode) {
  SimArgs a{};
  a.qhi = mode == CMVE_SIM_F16 ? q->h16 : q->hi;
  a.qlo = q->lo;
  a.ghi = mode == CMVE_SIM_F16 ? g->h16 : g->hi;
  a.glo = g->lo;
  a.ldk = q->d_pad;
  a.nq = (int)q->n;
  a.ng = (int)g->n;
  a.nblk_m = (int)(q->n_pad / BM);
  a.nblk_n = (int)(g->n_pad / BN);
  a.nk = (int)(q->d_pad / BK);
  return a;
}

}  // namespace cmve

using namespace cmve;

extern "C" int cmve_sim_store(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, float alpha,
                              float beta, void* out, int32_t out_dtype, int64_t ldo) {
  CMVE_REQUIRE(h, "cmve_sim_store: NULL handle");
  int st = validate_pair(q, g, mode, "cmve_sim_store");
  if (st) return st;
  CMVE_REQUIRE(out && ldo >= g->n, "cmve_sim_store: bad output");
  CMVE_REQUIRE(out_dtype == CMVE_F32 || out_dtype == CMVE_F64, "cmve_sim_store: out_dtype must be F32/F64");
  if (q->n == 0 || g->n == 0) return CMVE_OK;
  SimArgs a = make_args(q, g, mode);
  a.out = out;
  a.ldo = ldo;
  a.alpha = alpha;
  a.beta = beta;
  a.out_f64 = out_dtype == CMVE_F64;
  if (mode == CMVE_SIM_BF16) return launch_sim<CMVE_SIM_BF16, EPI_STORE>(a, h->stream);
  if (mode == CMVE_SIM_F16) return launch_sim<CMVE_SIM_F16, EPI_STORE>(a, h->stream);
  return launch_sim<CMVE_SIM_BF16X3, EPI_STORE>(a, h->stream);
}

// defined in rank.hip
namespace cmve {
int launch_fixup(hipStream_t stream, const cmve_rows_t* q, const cmve_rows_t* g, int32_t dirs, const double* row_sgt,
                 const double* col_sgt, int32_t* row_cnt, int32_t* col_cnt, const uint64_t* cand, int64_t cand_cap,
                 const int64_t* cand_count);
}

static int rank_args(const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, int32_t dirs, const float* row_hi,
                     const float* row_lo, const float* col_hi, const float* col_lo, int32_t* row_cnt, int32_t* col_cnt,
                     uint64_t* cand, int64_t cand_cap, int64_t* cand_count, SimArgs& a, const char* fn) {
  int st = validate_pair(q, g, mode, fn);
  if (st) return st;
  CMVE_REQUIRE((dirs & ~3) == 0 && dirs != 0, "%s: dirs must be a non-empty subset of ROW|COL", fn);
  if (dirs & CMVE_DIR_ROW) CMVE_REQUIRE(row_hi && row_lo && row_cnt, "%s: row arrays missing", fn);
  if (dirs & CMVE_DIR_COL) CMVE_REQUIRE(col_hi && col_lo && col_cnt, "%s: col arrays missing", fn);
  CMVE_REQUIRE(cand && cand_count && cand_cap >= 0, "%s: candidate buffer missing", fn);
  a = make_args(q, g, mode);
  if (dirs & CMVE_DIR_ROW) {
    a.row_hi = row_hi;
    a.row_lo = row_lo;
    a.row_cnt = row_cnt;
  }
  if (dirs & CMVE_DIR_COL) {
    a.col_hi = col_hi;
    a.col_lo = col_lo;
    a.col_cnt = col_cnt;
  }
  a.cand = (unsigned long long*)cand;
  a.cand_cap = cand_cap;
  a.cand_count = (unsigned long long*)cand_count;
  return CMVE_OK;
}

extern "C" int cmve_rank_mfma(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, int32_t dirs,
                              const float* row_hi, const float* row_lo, const float* col_hi, const float* col_lo,
                              int32_t* row_cnt, int32_t* col_cnt, uint64_t* cand, int64_t cand_cap,
                              int64_t* cand_count) {
  CMVE_REQUIRE(h, "cmve_rank_mfma: NULL handle");
  SimArgs a;
  int st = rank_args(q, g, mode, dirs, row_hi, row_lo, col_hi, col_lo, row_cnt, col_cnt, cand, cand_cap, cand_count,
                     a, "cmve_rank_mfma");
  if (st) return st;
  CMVE_HIP(hipMemsetAsync(cand_count, 0, sizeof(int64_t), h->stream));
  if (dirs & CMVE_DIR_ROW) CMVE_HIP(hipMemsetAsync(row_cnt, 0, sizeof(int32_t) * q->n_pad, h->stream));
  if (dirs & CMVE_DIR_COL) CMVE_HIP(hipMemsetAsync(col_cnt, 0, sizeof(int32_t) * g->n_pad, h->stream));
  if (q->n == 0 || g->n == 0) return CMVE_OK;
  if (mode == CMVE_SIM_BF16) return launch_sim<CMVE_SIM_BF16, EPI_RANK>(a, h->stream);
  if (mode == CMVE_SIM_F16) return launch_sim<CMVE_SIM_F16, EPI_RANK>(a, h->stream);
  return launch_sim<CMVE_SIM_BF16X3, EPI_RANK>(a, h->stream);
}

extern "C" int cmve_rank_fixup(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t dirs,
                               const double* row_sgt, const double* col_sgt, int32_t* row_cnt, int32_t* col_cnt,
                               const uint64_t* cand, int64_t cand_cap, const int64_t* cand_count) {
  CMVE_REQUIRE(h && q && g, "cmve_rank_fixup: NULL argument");
  CMVE_REQUIRE(q->d == g->d, "cmve_rank_fixup: dimension mismatch");
  CMVE_REQUIRE(q->raw && g->raw && q->inv_norm && g->inv_norm, "cmve_rank_fixup: raw rows / norms missing");
  if (dirs & CMVE_DIR_ROW) CMVE_REQUIRE(row_sgt && row_cnt, "cmve_rank_fixup: row arrays missing");
  if (dirs & CMVE_DIR_COL) CMVE_REQUIRE(col_sgt && col_cnt, "cmve_rank_fixup: col arrays missing");
  CMVE_REQUIRE(cand && cand_count, "cmve_rank_fixup: candidate buffer missing");
  if (q->n == 0 || g->n == 0) return CMVE_OK;
  return launch_fixup(h->stream, q, g, dirs, row_sgt, col_sgt, row_cnt, col_cnt, cand, cand_cap, cand_count);
}

extern "C" int cmve_rank_count(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, int32_t dirs,
                               const double* row_sgt, const float* row_hi, const float* row_lo, const double* col_sgt,
                               const float* col_hi, const float* col_lo, int32_t* row_cnt, int32_t* col_cnt,
                               uint64_t* cand, int64_t cand_cap, int64_t* cand_count) {
  if (dirs & CMVE_DIR_ROW) CMVE_REQUIRE(row_sgt, "cmve_rank_count: row_sgt missing");
  if (dirs & CMVE_DIR_COL) CMVE_REQUIRE(col_sgt, "cmve_rank_count: col_sgt missing");
  int st = cmve_rank_mfma(h, q, g, mode, dirs, row_hi, row_lo, col_hi, col_lo, row_cnt, col_cnt, cand, cand_cap,
                          cand_count);
  if (st) return st;
  return cmve_rank_fixup(h, q, g, dirs, row_sgt, col_sgt, row_cnt, col_cnt, cand, cand_cap, cand_count);
}

extern "C" int cmve_linear(cmve_handle_t h, const cmve_rows_t* x, const cmve_rows_t* w, int32_t mode, const float* bias,
                           const float* bn_scale, const float* bn_shift, const float* resid, int64_t ldr, int32_t relu,
                           float* out, int64_t ldo) {
  CMVE_REQUIRE(h, "cmve_linear: NULL handle");
  int st = validate_pair(x, w, mode, "cmve_linear");
  if (st) return st;
  CMVE_REQUIRE(out && ldo >= w->n, "cmve_linear: bad output");
  CMVE_REQUIRE((bn_scale == nullptr) == (bn_shift == nullptr), "cmve_linear: bn_scale and bn_shift go together");
  CMVE_REQUIRE(!resid || ldr >= w->n, "cmve_linear: bad residual leading dimension");
  if (x->n == 0 || w->n == 0) return CMVE_OK;
  SimArgs a = make_args(x, w, mode);
  a.out = out;
  a.ldo = ldo;
  a.bias = bias;
  a.bn_scale = bn_scale;
  a.bn_shift = bn_shift;
  a.resid = resid;
  a.ldr = ldr;
  a.relu = relu;
  if (mode == CMVE_SIM_BF16) return launch_sim<CMVE_SIM_BF16, EPI_LINEAR>(a, h->stream);
  if (mode == CMVE_SIM_F16) return launch_sim<CMVE_SIM_F16, EPI_LINEAR>(a, h->stream);
  return launch_sim<CMVE_SIM_BF16X3, EPI_LINEAR>(a, h->stream);
}
