// K4: N_q x N_g cosine-similarity GEMM on bf16 / fp16 MFMA (gfx950), with fused epilogues.
//
//   EPI_STORE  : out[i,j] = alpha * s_ij + beta            (cal_error / cal_simi / logits)
//   EPI_RANK   : per-row and per-column "score > threshold" counts + undecided-pair list
//                (the GT rank of LINAS-engine/util/metrics.py:137-147 without the matrix)
//   EPI_LINEAR : BN(resid + act(x.w + bias))               (MFC / Combiner projections)
//   EPI_BIAS   : x.w + bias (+ ReLU): EPI_LINEAR's common case as its own instantiation
//   EPI_TOPK   : the RANK epilogue with thresholds (+inf, tau): every s >= tau emitted as a
//                (score key, row, column) entry, bucketed by 256-row QUERY tile (topk.hip K13)
//
// Geometry (template WM x WN waves, each wave TM x 4 tiles of v_mfma_f32_16x16x32):
//   G128: 2 x 2 waves, 64 x 64 per wave  -> 128 x 128 block tile, 256 threads, 2 blocks / CU
//   G256: 2 x 4 waves, 128 x 64 per wave -> 256 x 256 block tile, 512 threads, 1 block / CU
// The 256^2 tile doubles the FLOP per staged byte (128 vs 64 FLOP/B), which a 128^2 tile
// cannot feed from L2 at the MFMA rate (~63 B/clk/CU needed vs ~56 available); G256 is the
// default for problems with >= 512 tiles (split-bf16 included: one bf16 GEMM over K' = 3K), G128 for small
// problems.  K step 64; staging by global_load_lds_dwordx4 (16 B / lane, 1 KiB per wave
// instruction) into a lane-linear LDS image, 2 stages; bank conflicts removed by an XOR
// swizzle applied to the GLOBAL source chunk (chunk ^ (row & 7)) and the matching
// ds_read_b128 address.  Grid: XCD-aware -- each XCD gets a contiguous range of the logical
// tile order, which walks 8 gallery tiles x all query tiles.
#include <algorithm>
#include <vector>

#include <hip/hip_ext.h>

#include "cmve_internal.h"

// Study knobs are compile-time only (make study NAME=x DEFS="-D..."): the product build reads no environment.
#ifndef CMVE_SIM_GN
#define CMVE_SIM_GN 8  // gallery tiles per tile-order group (GN = 2..16 measured within 2%)
#endif
#ifndef CMVE_SIM_GEO
#define CMVE_SIM_GEO 0  // 128: force G128; 2562: the 2-stage G256 loop
#endif
#ifndef CMVE_BATCH_GEO
#define CMVE_BATCH_GEO 0  // K14 batch rank tile: 1288 / 256128 / 64 / 12864 (see batch_geo_force)
#endif
#ifndef CMVE_EVAL_DBG
#define CMVE_EVAL_DBG 0  // K14 kernel studies: skip parts (results garbage) / 128: per-block stamps
#endif
#ifndef CMVE_EVAL_INLINE_L2
#define CMVE_EVAL_INLINE_L2 1  // 0: the level-2 re-score in a fix-up launch instead of inside the rank GEMM
#endif
#ifndef CMVE_EVAL_NO_L2
#define CMVE_EVAL_NO_L2 0  // 1: every band pair in fp64 inside the GEMM (no residual plane)
#endif
#ifndef CMVE_EVAL_L3_LIST
#define CMVE_EVAL_L3_LIST 0  // 1: one evaluation lists its level-3 pairs for the finish as batches do
#endif
#ifndef CMVE_L2_PIPE
#define CMVE_L2_PIPE 1  // K14 level-2 re-score: one pair per wave per step, the next pair's rows in flight (0: rounds
#endif                  // of CMVE_L2_P* pairs per wave, each round one round trip)
#ifndef CMVE_G64_KG
#define CMVE_G64_KG 2  // one K14 evaluation's G64 rank GEMM: K groups (2: split-K over two groups of 4 waves)
#endif
#ifndef CMVE_EPI_BOTH_ASM
#define CMVE_EPI_BOTH_ASM 1  // rank epilogue, both directions: hand-scheduled scoring (pair2_count_bits); 0: compiler's
#endif
#ifndef CMVE_EPI_T2V_DBL
#define CMVE_EPI_T2V_DBL 0  // rank epilogue, t2v only: col4_count_bits (band bits by doubling) instead of row4_count_bits
#endif
#ifndef CMVE_RING_KROT
#define CMVE_RING_KROT 0  // the batch ring: K-slice order rotated per tile (study)
#endif
#ifndef CMVE_RING_VGPR_STAGE
#define CMVE_RING_VGPR_STAGE 0  // the batch ring: K-tiles staged through registers instead of LDS-DMA (study)
#endif
#ifndef CMVE_RING_READS_FIRST
// ring loops: a K-tile's fragment reads all issued before its MFMAs (study: the batch rank GEMM alone 41.0 -> 38.4 us,
// one stream 8.5 -> 8.65e10, but three streams 1.26 -> 1.20e11 -- profiles/r06_ab_reads_first.txt)
#define CMVE_RING_READS_FIRST 0
#endif

namespace cmve {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int BK = 64;
constexpr int EPI_STORE = 0, EPI_RANK = 1, EPI_LINEAR = 2, EPI_TOPK = 3, EPI_BIAS = 4;
// epilogues that count / emit against per-row and per-column thresholds
constexpr bool epi_thr(int e) { return e == EPI_RANK || e == EPI_TOPK; }

struct SimArgs {
  const uint16_t* qhi;
  const uint16_t* qlo;
  const uint16_t* ghi;
  const uint16_t* glo;
  int64_t ldk;  // d_pad
  int nq, ng;
  int nblk_m, nblk_n;
  int nk;   // K-tiles of the MFMA loop (split-bf16: 3 x nk0, see plane_of)
  int nk0;  // K-tiles of one plane (d_pad / BK)
  int gn;  // gallery tiles per tile-order group
  // linear epilogue: v = acc + bias; act; + resid; v * bn_scale + bn_shift
  const float* bias;
  const float* bn_scale;
  const float* bn_shift;
  const float* resid;
  int64_t ldr;
  int relu;  // activation: 0 none, 1 ReLU, 2 QuickGELU, 3 sigmoid
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
  unsigned long long* cand;        // bucket storage (cand_layout): bucket b at cand + b * cap_b
  long long cand_cap;
  unsigned long long* cand_count;
  unsigned long long* bucket_cnt;  // per-bucket pair counters (head of the caller's buffer)
  long long cap_b;
  // rank thresholds derived in-kernel from the exact GT scores (K14): thr = dir-rounded sgt +- E(e_row,
  // err_max of the other set), the err_max reduced from the other set's per-row bounds at kernel start;
  // replaces row_hi / row_lo / col_hi / col_lo (which then only say which directions are on)
  int thr_gt;
  const double* row_sgt;
  const double* col_sgt;
  const float* q_err;  // per-row bounds of the mode's plane, [n_pad] (padding rows 0)
  const float* g_err;
  const unsigned* q_emax;  // err_max shards of the mode's plane, [EMAX_SHARDS] float bits each side
  const unsigned* g_emax;
  unsigned long long* dbg_stamps;  // kernel studies only: [tile][8] stamps, nullptr otherwise
  // K14: undecided pairs bucketed by 64 x 64 output tile (bucket (m0 >> 6) * nbn64 + (n0 >> 6)) instead of by
  // 256 gallery rows: a 1k x 1k evaluation otherwise sends every wave's slot reservation to one of 4 counters
  int tile_buckets;
  int nbn64;
  // K14: the first GT of every row / column (-1: none); the 2-stage / ring rank epilogues drop that GT pair
  // from the undecided list -- a GT item's score never exceeds its row's best GT score, so it is never counted
  const int* row_gt1;
  const int* col_gt1;
  // K14 at G64 (the ring kernel): the undecided pairs are re-scored in fp64 inside the epilogue (fixup_walk's
  // arithmetic, wave_cos64 on the raw rows) instead of being listed for a fix-up launch
  int fix_inline;
  int q_f64, g_f64;
  const void* q_raw;
  const void* g_raw;
  int64_t q_ld, g_ld, d;
  const double* q_inv;
  const double* g_inv;
  // K14 level-2 re-score (F16 rank path): the bf16 residual planes the prep wrote beside the fp16 planes (qhi /
  // ghi) and their per-row bounds; a band pair is decided from h16 + lo16 (lo16_elem) when its score clears the
  // GT score by the level-2 bound; the rest go to the level-3 list (EvalCommon::l3, re-scored in fp64 by the
  // finish), or are re-scored here when it is full.  nullptr: every pair in fp64 here
  int ovf_inline;  // K14 with a fix-up launch: a wave whose pairs overflow its bucket re-scores them itself
  const uint16_t* q_lo16;
  const uint16_t* g_lo16;
  const float* q_el;
  const float* g_el;
  unsigned* l3_count;
  unsigned long long* l3;
  int l3_cap;
};

// (L16Frag, l16_load, l16_partial: the level-2 re-score's fragments, cmve_internal.h)
// the wave's level-2 scores of P pairs (rows qr[p] of the query planes, gc[p] of the gallery planes), every
// load of all P pairs in flight before the sums; d_pad % 64 == 0 (a lane's 16 elements are all in or all out)
template <int P>
__device__ __forceinline__ void l16_scores(const SimArgs& a, const int64_t (&qr)[P], const int64_t (&gc)[P], int lane,
                                          double (&s2)[P]) {
#pragma unroll
  for (int p = 0; p < P; ++p) s2[p] = 0.0;
  for (int64_t k0 = 0; k0 < a.ldk; k0 += 1024) {
    const int64_t k = k0 + 16 * lane;
    if (k < a.ldk) {
      L16Frag fq[P], fg[P];
#pragma unroll
      for (int p = 0; p < P; ++p) {
        l16_load(a.qhi + qr[p] * a.ldk, a.q_lo16 + qr[p] * a.ldk, k, fq[p]);
        l16_load(a.ghi + gc[p] * a.ldk, a.g_lo16 + gc[p] * a.ldk, k, fg[p]);
      }
#pragma unroll
      for (int p = 0; p < P; ++p) s2[p] = l16_partial(fq[p], fg[p], s2[p]);
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
    for (int p = 0; p < P; ++p) s2[p] += __shfl_xor(s2[p], o, 64);
}

// bijective XCD remap (xcd_linear, cmve_internal.h) + grouped (GN gallery tiles x all query tiles) logical order
__device__ __forceinline__ void tile_grouped(int L, int nblk_m, int nblk_n, int GN, int& bm, int& bn);
__device__ __forceinline__ void tile_of_block(int bid, int nblk_m, int nblk_n, int GN, int& bm, int& bn) {
  tile_grouped(xcd_linear(bid, nblk_m * nblk_n), nblk_m, nblk_n, GN, bm, bn);
}
__device__ __forceinline__ void tile_grouped(int L, int nblk_m, int nblk_n, int GN, int& bm, int& bn) {
  const int group = L / (GN * nblk_m);
  const int within = L - group * (GN * nblk_m);
  const int gn = min(GN, nblk_n - group * GN);
  bm = within / gn;
  bn = group * GN + (within - bm * gn);
}

// the LDS image of a staged K-tile of KB (64 or 32) bf16/fp16 columns: row r at r * 2KB bytes, its 16-B chunk k in
// slot k ^ swz(r) -- conflict-free ds_read_b128 fragment reads (16 rows x one chunk per 16 lanes): 128-B rows
// (KB = 64, 8 chunks) XOR the row's low 3 bits; 64-B rows (KB = 32, 4 chunks, four rows per 256-B bank line) XOR
// bits 2-3, so rows r, r + 4, r + 8, r + 12 of one bank offset take four different slots
template <int KB>
__host__ __device__ constexpr int lds_swz(int r) {
  return KB == 64 ? (r & 7) : ((r >> 2) & 3);
}

// this lane's byte offset inside any staging wave-instruction of a KB-deep K-tile: one instruction's 64 lanes cover
// RPI whole rows, and the swizzle takes only a row's low bits (KB = 64: r & 7 with RPI = 8; KB = 32: (r >> 2) & 3
// with RPI = 16), so the offset is the same for every instruction of every wave -- computed once per kernel, the K
// loop's staging is scalar address math (per-instruction 64-bit lane address math cost ~60 VALU cycles x 8 per wave
// per K-tile in the batch ring)
template <int KB>
__device__ __forceinline__ uint32_t stage_lane_off(int64_t ldk, int lane) {
  constexpr int CPR = KB / 8;  // 16-B chunks per row
  const int r = lane / CPR, c = lane % CPR;
  return (uint32_t)(((int64_t)r * ldk + (c ^ lds_swz<KB>(r)) * 8) * 2);
}

// issue this wave's share of one ROWS x KB (bf16/fp16) plane: ROWS x 2KB / 1 KiB wave-instructions of 1 KiB; src,
// ldk, row0, k0 and wave are uniform (the block base is scalar; loff = stage_lane_off<KB>)
template <int ROWS, int NW, int KB = BK>
__device__ __forceinline__ void stage_plane(const uint16_t* __restrict__ src, int64_t ldk, int row0, int k0,
                                            char* lds_plane, int wave, uint32_t loff) {
  constexpr int CPR = KB / 8;    // 16-B chunks per row
  constexpr int RPI = 64 / CPR;  // rows per wave-instruction
  constexpr int PER_WAVE = ROWS / RPI / NW;
  static_assert(PER_WAVE * RPI * NW == ROWS, "plane rows must split evenly over the waves");
  static_assert(lds_swz<KB>(RPI) == 0 && lds_swz<KB>(RPI - 1) == lds_swz<KB>(2 * RPI - 1), "swizzle period");
  const char* blk = (const char*)(src + ((int64_t)row0 + wave * PER_WAVE * RPI) * ldk + k0);
#pragma unroll
  for (int it = 0; it < PER_WAVE; ++it)
    __builtin_amdgcn_global_load_lds((const void*)(blk + (int64_t)it * RPI * ldk * 2 + loff),
                                     (lds_void_t*)(lds_plane + (wave * PER_WAVE + it) * 1024), 16, 0, 0);
}

template <int KB = BK>
__device__ __forceinline__ s16x8_t read_frag(const char* plane, int row, int chunk) {
  return *(const s16x8_t*)(plane + row * (KB * 2) + ((chunk ^ lds_swz<KB>(row)) << 4));
}

// LDS atomic add in inline asm: the compiler drains vmcnt before any LDS write it emits while
// LDS-DMA loads are in flight (it cannot tell the staging buffers from the epilogue scratch), which
// made the first row count of every epilogue wait for the next tile's prefetch.  The callers
// order these adds with CMVE_BAR_LDS (lgkmcnt(0) + s_barrier) before anything reads the counters.
__device__ __forceinline__ void lds_add_u32_async(int* p, int v) {
  const uint32_t addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) int*)p;
  asm volatile("ds_add_u32 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

// sum over the 16 lanes of each DPP row (quad xor 1, xor 2, half-row mirror, row mirror): 4 VALU
__device__ __forceinline__ uint32_t row_sum16(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
  return v;
}

// One row's 4 scores (columns j = 0..3 of lane row R) against its thresholds, hand-scheduled:
// returns #{s > hi} (exact v_cmp; NaN never counts) and ORs the exact "lo <= s <= hi" bits into u at
// bit 4j + R (s >= lo and not s > hi: lo <= hi, or both NaN / +inf, for every threshold pair).  Every
// lane mask goes to its own SGPR pair and is read >= 4 instructions after it is written, so no wait
// states are needed (the compiler routed each compare through VCC with an s_nop before the reader).
template <int R>
__device__ __forceinline__ uint32_t row4_count_bits(float s0, float s1, float s2, float s3, float hi, float lo,
                                                    uint32_t& u) {
  uint32_t c, b0, b1, b2, b3;
  unsigned long long m0, m1, m2, m3, l0, l1, l2, l3, cc;
  asm("v_cmp_gt_f32_e64 %[m0], %[s0], %[hi]\n\t"
      "v_cmp_gt_f32_e64 %[m1], %[s1], %[hi]\n\t"
      "v_cmp_gt_f32_e64 %[m2], %[s2], %[hi]\n\t"
      "v_cmp_gt_f32_e64 %[m3], %[s3], %[hi]\n\t"
      "v_cmp_ge_f32_e64 %[l0], %[s0], %[lo]\n\t"
      "v_cmp_ge_f32_e64 %[l1], %[s1], %[lo]\n\t"
      "v_cmp_ge_f32_e64 %[l2], %[s2], %[lo]\n\t"
      "v_cmp_ge_f32_e64 %[l3], %[s3], %[lo]\n\t"
      "v_cndmask_b32_e64 %[c], 0, 1, %[m0]\n\t"
      "v_addc_co_u32_e64 %[c], %[cc], %[c], 0, %[m1]\n\t"
      "v_addc_co_u32_e64 %[c], %[cc], %[c], 0, %[m2]\n\t"
      "v_addc_co_u32_e64 %[c], %[cc], %[c], 0, %[m3]\n\t"
      "s_andn2_b64 %[l0], %[l0], %[m0]\n\t"
      "s_andn2_b64 %[l1], %[l1], %[m1]\n\t"
      "s_andn2_b64 %[l2], %[l2], %[m2]\n\t"
      "s_andn2_b64 %[l3], %[l3], %[m3]\n\t"
      "v_cndmask_b32_e64 %[b0], 0, 1, %[l0]\n\t"
      "v_cndmask_b32_e64 %[b1], 0, 1, %[l1]\n\t"
      "v_cndmask_b32_e64 %[b2], 0, 1, %[l2]\n\t"
      "v_cndmask_b32_e64 %[b3], 0, 1, %[l3]\n\t"
      "v_lshl_or_b32 %[u], %[b0], %[sh0], %[u]\n\t"
      "v_lshl_or_b32 %[u], %[b1], %[sh1], %[u]\n\t"
      "v_lshl_or_b32 %[u], %[b2], %[sh2], %[u]\n\t"
      "v_lshl_or_b32 %[u], %[b3], %[sh3], %[u]"
      : [c] "=&v"(c), [b0] "=&v"(b0), [b1] "=&v"(b1), [b2] "=&v"(b2), [b3] "=&v"(b3), [u] "+v"(u),
        [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3), [l0] "=&s"(l0), [l1] "=&s"(l1),
        [l2] "=&s"(l2), [l3] "=&s"(l3), [cc] "=&s"(cc)
      : [s0] "v"(s0), [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [hi] "v"(hi), [lo] "v"(lo), [sh0] "n"(R),
        [sh1] "n"(4 + R), [sh2] "n"(8 + R), [sh3] "n"(12 + R));
  return c;
}

// Both directions at once (the K14 evaluation's shape): two scores sa, sb of one column block (rows ra, rb of the
// lane's four) against their row thresholds (hia, loa), (hib, lob) and the column's (chi, clo).  Adds the exact
// counts #{s > hi} to ca, cb (row) and cc (column) and appends the exact band bits "lo <= s <= hi" (s >= lo and not
// s > hi: lo <= hi, or both NaN / +inf) to urow / ucol by doubling -- u = 2u + bit is ONE v_addc with the lane mask
// as carry-in, so the callers feed bits most significant first (j = 3..0, then r = 3..0: bit j * 4 + r).  8 VALU
// + 2 SALU per score (the compiler's form of the same tests: ~18 VALU).  Every lane mask has its own SGPR pair and
// is read >= 4 instructions after it is written (row4_count_bits' rule).
__device__ __forceinline__ void pair2_count_bits(float sa, float sb, float hia, float loa, float hib, float lob,
                                                 float chi, float clo, uint32_t& ca, uint32_t& cb, uint32_t& cc,
                                                 uint32_t& urow, uint32_t& ucol) {
  unsigned long long ma, mb, na, nb, la, lb, ka, kb, cy;
  asm("v_cmp_gt_f32_e64 %[ma], %[sa], %[hia]\n\t"
      "v_cmp_gt_f32_e64 %[mb], %[sb], %[hib]\n\t"
      "v_cmp_gt_f32_e64 %[na], %[sa], %[chi]\n\t"
      "v_cmp_gt_f32_e64 %[nb], %[sb], %[chi]\n\t"
      "v_cmp_ge_f32_e64 %[la], %[sa], %[loa]\n\t"
      "v_cmp_ge_f32_e64 %[lb], %[sb], %[lob]\n\t"
      "v_cmp_ge_f32_e64 %[ka], %[sa], %[clo]\n\t"
      "v_cmp_ge_f32_e64 %[kb], %[sb], %[clo]\n\t"
      "v_addc_co_u32_e64 %[ca], %[cy], %[ca], 0, %[ma]\n\t"
      "v_addc_co_u32_e64 %[cb], %[cy], %[cb], 0, %[mb]\n\t"
      "v_addc_co_u32_e64 %[cc], %[cy], %[cc], 0, %[na]\n\t"
      "v_addc_co_u32_e64 %[cc], %[cy], %[cc], 0, %[nb]\n\t"
      "s_andn2_b64 %[la], %[la], %[ma]\n\t"
      "s_andn2_b64 %[lb], %[lb], %[mb]\n\t"
      "s_andn2_b64 %[ka], %[ka], %[na]\n\t"
      "s_andn2_b64 %[kb], %[kb], %[nb]\n\t"
      "v_addc_co_u32_e64 %[ur], %[cy], %[ur], %[ur], %[la]\n\t"
      "v_addc_co_u32_e64 %[ur], %[cy], %[ur], %[ur], %[lb]\n\t"
      "v_addc_co_u32_e64 %[uc], %[cy], %[uc], %[uc], %[ka]\n\t"
      "v_addc_co_u32_e64 %[uc], %[cy], %[uc], %[uc], %[kb]"
      : [ca] "+v"(ca), [cb] "+v"(cb), [cc] "+v"(cc), [ur] "+v"(urow), [uc] "+v"(ucol), [ma] "=&s"(ma),
        [mb] "=&s"(mb), [na] "=&s"(na), [nb] "=&s"(nb), [la] "=&s"(la), [lb] "=&s"(lb), [ka] "=&s"(ka),
        [kb] "=&s"(kb), [cy] "=&s"(cy)
      : [sa] "v"(sa), [sb] "v"(sb), [hia] "v"(hia), [loa] "v"(loa), [hib] "v"(hib), [lob] "v"(lob), [chi] "v"(chi),
        [clo] "v"(clo));
}

// t2v only (the gallery shape): the four scores of one column block (rows r = 3..0 of the lane's four) against
// their row thresholds; the counts go to c3..c0 and the band bits are appended to u by doubling (bit j * 4 + r, most
// significant first, as pair2_count_bits): 4 VALU + 1 SALU per score (row4_count_bits: 5 + 1)
__device__ __forceinline__ void col4_count_bits(float s3, float s2, float s1, float s0, const f32x4_t& hi,
                                                const f32x4_t& lo, uint32_t& c3, uint32_t& c2, uint32_t& c1,
                                                uint32_t& c0, uint32_t& u) {
  unsigned long long m3, m2, m1, m0, l3, l2, l1, l0, cy;
  asm("v_cmp_gt_f32_e64 %[m3], %[s3], %[h3]\n\t"
      "v_cmp_gt_f32_e64 %[m2], %[s2], %[h2]\n\t"
      "v_cmp_gt_f32_e64 %[m1], %[s1], %[h1]\n\t"
      "v_cmp_gt_f32_e64 %[m0], %[s0], %[h0]\n\t"
      "v_cmp_ge_f32_e64 %[l3], %[s3], %[o3]\n\t"
      "v_cmp_ge_f32_e64 %[l2], %[s2], %[o2]\n\t"
      "v_cmp_ge_f32_e64 %[l1], %[s1], %[o1]\n\t"
      "v_cmp_ge_f32_e64 %[l0], %[s0], %[o0]\n\t"
      "v_addc_co_u32_e64 %[c3], %[cy], %[c3], 0, %[m3]\n\t"
      "v_addc_co_u32_e64 %[c2], %[cy], %[c2], 0, %[m2]\n\t"
      "v_addc_co_u32_e64 %[c1], %[cy], %[c1], 0, %[m1]\n\t"
      "v_addc_co_u32_e64 %[c0], %[cy], %[c0], 0, %[m0]\n\t"
      "s_andn2_b64 %[l3], %[l3], %[m3]\n\t"
      "s_andn2_b64 %[l2], %[l2], %[m2]\n\t"
      "s_andn2_b64 %[l1], %[l1], %[m1]\n\t"
      "s_andn2_b64 %[l0], %[l0], %[m0]\n\t"
      "v_addc_co_u32_e64 %[u], %[cy], %[u], %[u], %[l3]\n\t"
      "v_addc_co_u32_e64 %[u], %[cy], %[u], %[u], %[l2]\n\t"
      "v_addc_co_u32_e64 %[u], %[cy], %[u], %[u], %[l1]\n\t"
      "v_addc_co_u32_e64 %[u], %[cy], %[u], %[u], %[l0]"
      : [c3] "+v"(c3), [c2] "+v"(c2), [c1] "+v"(c1), [c0] "+v"(c0), [u] "+v"(u), [m3] "=&s"(m3), [m2] "=&s"(m2),
        [m1] "=&s"(m1), [m0] "=&s"(m0), [l3] "=&s"(l3), [l2] "=&s"(l2), [l1] "=&s"(l1), [l0] "=&s"(l0),
        [cy] "=&s"(cy)
      : [s3] "v"(s3), [s2] "v"(s2), [s1] "v"(s1), [s0] "v"(s0), [h3] "v"(hi[3]), [h2] "v"(hi[2]), [h1] "v"(hi[1]),
        [h0] "v"(hi[0]), [o3] "v"(lo[3]), [o2] "v"(lo[2]), [o1] "v"(lo[1]), [o0] "v"(lo[0]));
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

template <int WM, int WN, int TM>
struct Geo {
  static constexpr int TN = 4;
  static constexpr int NW = WM * WN;
  static constexpr int NT = NW * 64;
  static constexpr int BM = WM * TM * 16;
  static constexpr int BN = WN * TN * 16;
};

// staged bytes per K-tile: one plane per operand; the 2-stage G128 loop stages both planes of a
// split-bf16 operand per K-tile, the phased G256 loop walks the planes along K (plane_of)
template <int MODE, int BM, int BN, bool PHASED, int KB = BK>
constexpr size_t stage_bytes() {
  return (size_t)((MODE == CMVE_SIM_BF16X3 && !PHASED) ? 2 : 1) * (BM + BN) * KB * 2;
}

// the ring loop's geometries (G64, 128 x 64 and the 8-wave 128 x 128 of the batches); the others take the 2-stage
// loop (G128) or the phased G256 schedule
template <int BM, int BN, bool PHASED, int NW = 4>
constexpr bool is_ring() {
  return !PHASED && (((BN == 64 || (BM == 128 && BN == 128 && NW == 8)) && (BM == 64 || BM == 128)) ||
                     (BM == 256 && BN == 128 && NW == 8));
}
// the K14 batches' 256 x 128 tiles (one block of 8 waves of 64 x 64 per CU, up to 256 VGPRs)
template <int BM, int BN>
constexpr bool is_big_ring() {
  return BM == 256 && BN == 128;
}

// K-tile depth of a ring geometry's stages: the batches' 8-wave 128 x 128 ring stages 32-deep K-tiles
// (CMVE_BATCH_KB): at the same LDS, twice as many stages -- three K-tiles in flight instead of one, for a main loop
// that waits on L2 / Infinity-Cache latency (the stamps: 0.95 us per 64-deep K-tile against ~0.3 us of MFMAs)
#ifndef CMVE_BATCH_KB
#define CMVE_BATCH_KB 64
#endif
template <int BM, int BN, bool PHASED, int NW>
constexpr int ring_kb() {
  return (!PHASED && BM == 128 && BN == 128 && NW == 8) ? CMVE_BATCH_KB : BK;
}

// staging ring depth of the 2-stage (non-phased) loop: the G64 tiles of small problems keep NS - 1
// K-tiles in flight (a 1k x 1k x 1024 GEMM is latency-bound: with 2 stages every one of its 16 K-tiles
// exposed a full L2 / Infinity-Cache round trip, ~1.2 us each against ~0.1 us of MFMAs).  4 stages
// (64 KiB of LDS) rather than 8: a G64 block is bound by its 2 waves ISSUING the LDS-DMA pieces
// (8 per wave per K-tile, ~2.7 us for the first 7 K-tiles of an 8-deep ring in the stamps), so a deeper
// ring gains nothing alone, while 64 KiB lets two evaluations' rank GEMMs share a CU (two HIP streams:
// 31.0 -> 26.6 us per evaluation, tools/eval_pipe.py)
// The K14 batches' rings (cmve_eval_batch_*): 128 x 128 with 8 waves, 2 stages of 32 KiB -- two blocks per CU
// (<= 128 VGPRs: CMVE_BATCH_WPE), so one block's level-2 re-score round trips run under the other's main loop
// (round 4: rank GEMM 52 -> 38 us per batch of 8, headline 9.9e10 -> 1.11e11 against 3 stages of one block per
// CU) -- and 128 x 64 (split-bf16), 3 stages of 24 KiB
template <int MODE, int BM, int BN, bool PHASED, int NW = 4>
constexpr int ring_stages() {
#ifndef CMVE_G64_STAGES
#define CMVE_G64_STAGES 4
#endif
#ifndef CMVE_G128R_STAGES
#define CMVE_G128R_STAGES 2
#endif
  // (64 x 64, 128 x 64 and the 8-wave 128 x 128; the 4-wave G128 of mid-size problems keeps its 2-stage loop)
#ifndef CMVE_G256R_STAGES
#define CMVE_G256R_STAGES 3
#endif
  if (!PHASED && is_big_ring<BM, BN>() && NW == 8) return CMVE_G256R_STAGES;  // (3 x 48 KiB: one block per CU)
  // the batches' 128 x 128: CMVE_G128R_STAGES x 64-deep K-tiles of LDS, as twice as many 32-deep stages with
  // CMVE_BATCH_KB = 32 (ring_kb)
  return (PHASED || (BN != 64 && !(BM == 128 && BN == 128 && NW == 8)) || (BM != 64 && BM != 128))
             ? 2
             : (BM == 64 ? CMVE_G64_STAGES : CMVE_G128R_STAGES * (BK / ring_kb<BM, BN, PHASED, NW>()));
}

// the K-tile depth a kernel instantiation stages: ring_kb, but the 4-wave 128 x 128 batch ring takes CMVE_BATCH4_KB
// (32: a 32 KiB two-stage ring, three blocks per CU fit the LDS -- a study)
#ifndef CMVE_BATCH4_KB
#define CMVE_BATCH4_KB 64
#endif
template <int MODE, int BM, int BN, bool PHASED, int NW, bool BATCH>
constexpr int kernel_kb() {
  return (BATCH && !PHASED && BM == 128 && BN == 128 && NW == 4 && MODE != CMVE_SIM_BF16X3) ? CMVE_BATCH4_KB
                                                                                            : ring_kb<BM, BN, PHASED, NW>();
}

// LDS of the staging buffers of a non-persistent geometry (the launchers' dynamic shared memory)
template <int MODE, int BM, int BN, bool PHASED, int NW>
constexpr size_t ring_lds_bytes() {
  return ring_stages<MODE, BM, BN, PHASED, NW>() * stage_bytes<MODE, BM, BN, PHASED, ring_kb<BM, BN, PHASED, NW>()>();
}

#ifdef CMVE_DBG_STAMPS  // diagnostic build only: per-block s_memtime stamps into the (unused) candidate list
#define CMVE_STAMP(k) \
  if (threadIdx.x == 0) a.bucket_cnt[(size_t)tile * 8 + (k)] = __builtin_amdgcn_s_memtime()
#else  // kernel studies of the K14 evaluation (CMVE_EVAL_DBG & 128): s_memrealtime into SimArgs::dbg_stamps
// (the 2-stage / ring loops only: the persistent G256 kernel is compiled without them -- the extra
// scalar branches and stores cost it SGPR spills at the 256-VGPR cap)
#define CMVE_STAMP(k) \
  if constexpr (!PHASED) {  \
    if (a.dbg_stamps && threadIdx.x == 0) gst(a.dbg_stamps + (size_t)tile * 8 + (k), __builtin_amdgcn_s_memrealtime()); \
  }
#endif

// Split-bf16 (BF16X3) in the phased G256 loop: ONE bf16 GEMM over K' = 3K whose K'-tile 3t + p
// stages K-tile t of plane pair p = 0 (A lo, B hi), 1 (A hi, B lo), 2 (A hi, B hi) -- every
// product of the split once (n = 3 d).  The G128 loop stages all four planes of
// K-tile t and issues the same three pairs in the same order, so both geometries accumulate
// every output element in the identical MFMA sequence (bit-identical results across shapes).
__device__ __forceinline__ void plane_of(int tp, bool& a_lo, bool& b_lo, int& kt) {
  kt = tp / 3;
  const int p = tp - 3 * kt;
  a_lo = p == 0;
  b_lo = p == 1;
}

// Barrier for LDS hand-offs only: unlike __syncthreads it does not drain vmcnt, so loads issued
// for the next tile stay in flight across the epilogue's barriers.
#define CMVE_BAR_LDS() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

// Epilogue scratch as its own (static) LDS object: the staging buffers are the dynamic object that
// the LDS-DMA loads write, and the compiler orders an LDS access after in-flight LDS-DMA (vmcnt(0))
// only when it may alias that object -- with one shared dynamic object, the first epilogue LDS op
// drained the next tile's prefetch.
#ifndef CMVE_INL_LIST
#define CMVE_INL_LIST 1024
#endif
template <int BM, int BN, bool RANK, bool INL = false>
struct EpiLds {
  int rc[BM];
  int cc[BN];
  float thr[2 * (BM + BN)];  // [0,BM) row_hi, [BM,BM+BN) col_hi, then the lo halves
  double sgt[INL ? BM + BN : 1];  // inline fix-up (G64 K14): the rows' / columns' exact GT scores
  uint32_t list[INL ? CMVE_INL_LIST : 1];  // inline fix-up: the tile's undecided pairs (lr | lc << 8 | flags << 16)
  int wtot[INL ? 16 : 1];         // inline fix-up: per-wave pair counts
};
template <int BM, int BN, bool INL>
struct EpiLds<BM, BN, false, INL> {
  int rc[1], cc[1];
  float thr[1];
  double sgt[1];
  uint32_t list[1];
  int wtot[1];
};

#ifndef CMVE_G64_BLOCKS
#define CMVE_G64_BLOCKS 2
#endif
#ifndef CMVE_BATCH_FIX1
#define CMVE_BATCH_FIX1 1
#endif
#ifndef CMVE_L2_P
#define CMVE_L2_P 1  // K14 level-2 re-score: pairs per wave in flight at once (2: 128+ VGPRs, spills at 4 waves per SIMD)
#endif
#ifndef CMVE_L2_P_BIG
#define CMVE_L2_P_BIG 2  // the same for the batches' 256 x 128 tiles (one 8-wave block per CU: registers to spare)
#endif
#ifndef CMVE_L2_P_ONE
#define CMVE_L2_P_ONE 2  // the same for one evaluation's G64 rank GEMM (4 waves, ~6 listed pairs per tile: one round)
#endif
// BATCH: one launch over a batch of same-shaped problems (cmve_eval_batch_*): the block picks the problem's
// argument block in `tab` (see batch_item below); otherwise `tab` is unused
#ifndef CMVE_BATCH_WPE
#define CMVE_BATCH_WPE 4  // the batch ring kernels: waves per SIMD the register budget must allow (<= 128 VGPRs)
#endif
#ifndef CMVE_BATCH4_WPE
// the default 4-wave 128 x 128 batch tile: 3 waves per SIMD (<= 168 VGPRs) -- two GEMM blocks per CU and a wave of
// another stream's prep beside them on every SIMD (the product kernel needs 152)
#define CMVE_BATCH4_WPE 3
#endif
// KG = 2 (one K14 evaluation's G64 rank GEMM, sim_kernel_kg2): two groups of WM x WN waves, each streaming half of
// the K-tiles through a ring of its own; the second group's partial sums are added to the first's through LDS
// before the epilogue (every output element: two fp32 MFMA chains of d/2 then one fp32 add -- inside the same error
// bound, fewer roundings than one chain), and both groups share the level-2 re-score
template <int MODE, int EPI, int WM, int WN, int TM, bool PHASED, bool BATCH = false, int KG = 1>
__global__ __launch_bounds__(WM * WN * 64 * KG,
                            KG > 1 ? 1
                                   : (BATCH ? (is_big_ring<WM * TM * 16, WN * 64>()
                                                   ? 2
                                                   : (WM * WN == 4 ? (MODE == CMVE_SIM_BF16X3 ? 2 : CMVE_BATCH4_WPE)
                                                                   : CMVE_BATCH_WPE))
                                            : ((WM * TM * 16 == 64 && WN == 1) ? CMVE_G64_BLOCKS : 2)))
void sim_kernel(
    SimArgs a_arg, const SimArgs* __restrict__ tab) {
  // a batch's blocks: the (evaluation, tile) pairs in evaluation-major order, cut into 8 contiguous ranges, one per
  // XCD -- an XCD works through one or two evaluations at a time (a 1k-A evaluation's fp16 planes are 4 MB, its
  // L2's size), not a slice of every evaluation in flight (L2 hit rate 61% that way)
  int batch_item = 0, batch_tile = 0;
  if constexpr (BATCH) {
    const int per = (int)gridDim.x;
    const int L = xcd_linear((int)(blockIdx.y * gridDim.x + blockIdx.x), per * (int)gridDim.y);
    batch_item = L / per;
    batch_tile = L - batch_item * per;
  }
  const SimArgs& a = BATCH ? tab[batch_item] : a_arg;
  using G = Geo<WM, WN, TM>;
  constexpr int BM = G::BM, BN = G::BN, TN = G::TN, NT = G::NT, NW = G::NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KB = kernel_kb<MODE, BM, BN, PHASED, NW, BATCH>();  // K-tile depth of the staging buffers
  constexpr int STAGE_BYTES = (int)stage_bytes<MODE, BM, BN, PHASED, KB>();
  constexpr int NS = ring_stages<MODE, BM, BN, PHASED, NW>();
  constexpr int A_BYTES = BM * KB * 2, B_BYTES = BN * KB * 2;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably uniform: scalar M0 / soffset
  // KG = 2: group = which half of K this wave streams, lw = its wave within the group (the output layout)
  constexpr int NWT = NW * KG, NTT = NT * KG;
  const int group = KG > 1 ? wave / NW : 0, lw = wave - group * NW;
  const int wr = lw / WN, wc = lw % WN;
  // tiles: the phased (G256) kernel is persistent -- one block per CU walks tile, tile + gridDim.x,
  // ... (same XCD, same XCD-local order as a one-tile-per-block grid); the G128 grid is one tile each
  const int ntiles = a.nblk_m * a.nblk_n;
  int tile = BATCH ? batch_tile : (int)blockIdx.x;
  if (tile >= ntiles) return;  // (a grid / argument mismatch ends here instead of in a wild tile walk)
  int m0, n0;
  auto tile_origin = [&](int t, int& mo, int& no) {
    int bm_, bn_;
    if constexpr (BATCH) tile_grouped(t, a.nblk_m, a.nblk_n, a.gn, bm_, bn_);  // (the XCD split is above)
    else tile_of_block(t, a.nblk_m, a.nblk_n, a.gn, bm_, bn_);
    mo = bm_ * BM;
    no = bn_ * BN;
  };
  tile_origin(tile, m0, n0);
  CMVE_STAMP(0);
#ifdef CMVE_DBG_STAMPS  // where the block ran: XCC_ID (hwreg 20) << 32 | HW_ID (hwreg 4)
  if (threadIdx.x == 0)
    a.bucket_cnt[(size_t)tile * 8 + 7] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                                         (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);
#endif

  // the G64 ring rank kernel re-scores its undecided pairs itself when the K14 host asks (SimArgs::fix_inline)
  // (the batches' default 128 x 128 tiles on 4 waves of 64 x 64 take the ring loop too)
  constexpr bool RING = is_ring<BM, BN, PHASED, NW>() || (BATCH && BM == 128 && BN == 128 && NW == 4);
  constexpr bool INL = EPI == EPI_RANK && RING;
  __shared__ EpiLds<BM, BN, epi_thr(EPI), INL> epi;
  double sgt_pub = 0.0;  // INL: this thread's row / column GT score (tid < BM + BN), published with the thresholds
  int* lds_rc = epi.rc;
  int* lds_cc = epi.cc;
  float* lds_thr = epi.thr;
  float thr_hi_v = __builtin_nanf(""), thr_lo_v = __builtin_nanf("");
  // a tile's thresholds are fetched when its loads are issued and published to LDS in its
  // epilogue: the epilogue must not wait on HBM (8 dependent loads per wave there cost ~28%)
  // K14: the other set's err_max, folded once per block from the prep's shards (the max over real rows
  // of the per-row bounds, NaN dropped, as err_max_kernel computes it); the thresholds then follow
  // gt_thr_kernel's rule per row / column
  float qmax_v = 0.f, gmax_v = 0.f;
  auto reduce_err_max = [&]() {  // fold the prep's err_max shards (uniform addresses: scalar loads)
    unsigned mq = 0u, mg = 0u;
#pragma unroll
    for (int k = 0; k < EVAL_EMAX_SHARDS; ++k) {
      mq = max(mq, a.q_emax[k]);
      mg = max(mg, a.g_emax[k]);
    }
    qmax_v = __uint_as_float(mq);
    gmax_v = __uint_as_float(mg);
  };
  auto thr_of = [&](double sgt, float e, float emax_other, float& hi, float& lo) {
    // NaN (no GT, padding) or +inf (every GT NaN): never counted
    const double E = score_error_bound((double)e, (double)emax_other, a.ldk, MODE);
    hi = sgt < INFINITY ? f32_round_up(sgt + E) : INFINITY;
    lo = sgt < INFINITY ? f32_round_down(sgt - E) : INFINITY;
  };
  auto fetch_thr = [&](int mo, int no, float& hi, float& lo) {
    hi = lo = __builtin_nanf("");
    if (tid < BM) {
      if (a.row_hi) {
        if (!PHASED && a.thr_gt) thr_of(gld(a.row_sgt + mo + tid), gld(a.q_err + mo + tid), gmax_v, hi, lo);
        else {
          hi = gld(a.row_hi + mo + tid);
          lo = gld(a.row_lo + mo + tid);
        }
      }
    } else if (tid < BM + BN && a.col_hi) {
      if (!PHASED && a.thr_gt) thr_of(gld(a.col_sgt + no + tid - BM), gld(a.g_err + no + tid - BM), qmax_v, hi, lo);
      else {
        hi = gld(a.col_hi + no + tid - BM);
        lo = gld(a.col_lo + no + tid - BM);
      }
    }
  };
  // EPI_BIAS / EPI_LINEAR: the tile's bias (and BN) columns are fetched with its loads too
  constexpr bool EPI_COLS = EPI == EPI_BIAS || EPI == EPI_LINEAR;
  constexpr int NCV = EPI == EPI_LINEAR ? 3 : 1;  // bias, bn_scale, bn_shift
  float colv[NCV][TN];
  auto fetch_cols = [&](int no, float (*cv)[TN]) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = no + wc * (TN * 16) + j * 16 + (lane & 15);
      const bool ok = col < a.ng;
      cv[0][j] = (a.bias && ok) ? a.bias[col] : 0.f;
      if constexpr (NCV == 3) {
        cv[1][j] = (a.bn_scale && ok) ? a.bn_scale[col] : 1.f;
        cv[2][j] = (a.bn_shift && ok) ? a.bn_shift[col] : 0.f;
      }
    }
  };
  if constexpr (EPI_COLS) fetch_cols(n0, colv);
  if constexpr (epi_thr(EPI)) {
    static_assert(NT >= BM + BN, "one threshold pair per thread (threads past BM + BN hold none)");
    for (int t = tid; t < BM + BN; t += NTT) lds_rc[t] = 0;  // later tiles: reset by the flush
    // K14 thresholds need the block's err_max reduction first: the 2-stage / ring loops do both after
    // issuing their first loads (below).  The persistent G256 kernel never derives them (cmve_eval_ranks
    // writes them with eval_thr_kernel first): the derivation's code alone cost it 18% (SGPR spills at
    // the 256-VGPR cap, 3.86 -> 4.56 ms at 16,384 x 131,072)
    if (PHASED || !a.thr_gt) fetch_thr(m0, n0, thr_hi_v, thr_lo_v);
  }

  // the staging operands held in registers: a batch's `a` lives in device memory, and the compiler re-read these
  // fields (a scalar round trip) around the LDS-DMA issues of every K-tile
  const uint16_t* const st_qhi = a.qhi;
  const uint16_t* const st_ghi = a.ghi;
  const uint16_t* const st_qlo = MODE == CMVE_SIM_BF16X3 ? a.qlo : nullptr;
  const uint16_t* const st_glo = MODE == CMVE_SIM_BF16X3 ? a.glo : nullptr;
  const int64_t st_ldk = a.ldk;
  const uint32_t st_loff = stage_lane_off<KB>(st_ldk, lane);
  auto stage = [&](int t, int s) {
#ifdef CMVE_DBG_NOLOAD
    return;
#endif
    char* base = smem + (group * NS + s) * STAGE_BYTES;  // (KG = 2: each group's ring of its own)
    const int k0 = t * KB;
    stage_plane<BM, NW, KB>(st_qhi, st_ldk, m0, k0, base, lw, st_loff);
    stage_plane<BN, NW, KB>(st_ghi, st_ldk, n0, k0, base + A_BYTES, lw, st_loff);
    if (MODE == CMVE_SIM_BF16X3) {
      stage_plane<BM, NW, KB>(st_qlo, st_ldk, m0, k0, base + A_BYTES + B_BYTES, lw, st_loff);
      stage_plane<BN, NW, KB>(st_glo, st_ldk, n0, k0, base + 2 * A_BYTES + B_BYTES, lw, st_loff);
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // K14 (2-stage / ring rank kernels): the first GT of this lane's rows (i, r) and columns (j), fetched with
  // the thresholds; the epilogue clears those GT pairs' band bits (a GT pair is never counted: 1,000 of a
  // 1k-A evaluation's ~1,300 undecided t2v pairs are the GT pairs themselves)
  constexpr bool GT_SKIP = !PHASED && EPI == EPI_RANK;
  int gt_row[GT_SKIP ? TM : 1][4], gt_col[GT_SKIP ? TN : 1];
#pragma unroll
  for (int i = 0; i < (GT_SKIP ? TM : 1); ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) gt_row[i][r] = -1;
#pragma unroll
  for (int j = 0; j < (GT_SKIP ? TN : 1); ++j) gt_col[j] = -1;
  auto fetch_gt1 = [&]() {
    if constexpr (GT_SKIP) {
      const int rb = m0 + wr * (TM * 16) + (lane >> 4) * 4, cb = n0 + wc * (TN * 16) + (lane & 15);
      if (a.row_gt1)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) gt_row[i][r] = gld(a.row_gt1 + rb + i * 16 + r);  // (n_pad entries)
      if (a.col_gt1)
#pragma unroll
        for (int j = 0; j < TN; ++j) gt_col[j] = gld(a.col_gt1 + cb + j * 16);
    }
  };

  auto epilogue = [&]() {
  #ifdef CMVE_DBG_NOEPI  // diagnostic build only: main loop without any epilogue (results are garbage)
  #pragma unroll
    for (int i = 0; i < TM; ++i)
  #pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  #endif
    // ---------------- epilogues ----------------
    // accumulator element (i, j, r): row = m0 + wr*TM*16 + i*16 + (lane>>4)*4 + r,
    //                                col = n0 + wc*TN*16 + j*16 + (lane&15)
    const int rbase = m0 + wr * (TM * 16) + (lane >> 4) * 4;
    const int cbase = n0 + wc * (TN * 16) + (lane & 15);

    if constexpr (EPI == EPI_BIAS) {
      // bias (+ ReLU) only: a separate instantiation, so the general form's act / resid / BN
      // arguments do not hold scalar registers through the main loop (that one spills SGPRs), and
      // the bias columns arrive with the tile's loads (bias_v) instead of an HBM wait in here,
      // which would also wait for the next tile's staging loads already in flight
      const bool relu = a.relu == 1;
      float* outp = (float*)a.out;
  #pragma unroll
      for (int i = 0; i < TM; ++i)
  #pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rbase + i * 16 + r;
          if (row >= a.nq) continue;
  #pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = cbase + j * 16;
            const float v = acc[i][j][r] + colv[0][j];
            if (col < a.ng) outp[(int64_t)row * a.ldo + col] = relu ? fmaxf(v, 0.f) : v;
          }
        }
    } else if constexpr (EPI == EPI_LINEAR) {
      const float* bj = colv[0];
      const float* sj = colv[NCV - 1 > 0 ? 1 : 0];
      const float* hj = colv[NCV - 1 > 0 ? 2 : 0];
  #pragma unroll
      for (int i = 0; i < TM; ++i)
  #pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rbase + i * 16 + r;
          if (row >= a.nq) continue;
  #pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = cbase + j * 16;
            if (col >= a.ng) continue;
            float v = acc[i][j][r] + bj[j];
            if (a.relu == 1) v = fmaxf(v, 0.f);                         // ReLU
            else if (a.relu == 2) v = v / (1.f + expf(-1.702f * v));  // QuickGELU x*sigmoid(1.702x)
            else if (a.relu == 3) v = 1.f / (1.f + expf(-v));         // Sigmoid
            if (a.resid) v = a.resid[(int64_t)row * a.ldr + col] + v;
            if (a.bn_scale) v = v * sj[j] + hj[j];
            ((float*)a.out)[(int64_t)row * a.ldo + col] = v;
          }
        }
    } else if constexpr (EPI == EPI_STORE) {
  #pragma unroll
      for (int i = 0; i < TM; ++i)
  #pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rbase + i * 16 + r;
          if (row >= a.nq) continue;
  #pragma unroll
          for (int j = 0; j < TN; ++j) {
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
      // thresholds from LDS; a disabled direction holds NaN, which no comparison passes (not even s = +inf)
      if (tid < BM + BN) {
        lds_thr[tid] = thr_hi_v;
        lds_thr[BM + BN + tid] = thr_lo_v;
        if constexpr (INL) epi.sgt[tid] = sgt_pub;
      }
      CMVE_BAR_LDS();
      CMVE_STAMP(4);
      const float* l_rhi = lds_thr + (rbase - m0);
      const float* l_rlo = lds_thr + BM + BN + (rbase - m0);
      float chi[TN], clo[TN];
  #pragma unroll
      for (int j = 0; j < TN; ++j) {
        chi[j] = lds_thr[BM + (cbase - n0) + j * 16];
        clo[j] = lds_thr[BM + BN + BM + (cbase - n0) + j * 16];
      }
      // Branch-free scoring pass: per score only compares and bit packing.  Undecided pairs are
      // recorded as bits (per i: bit j*4+r = row-undecided, bit 16+j*4+r = column-undecided) and
      // emitted afterwards with ONE LDS atomic per wave; a per-score atomic with exec-mask
      // branches cost ~40% of the block (s_memtime stamps, tools/kbench.py KB_STAMPS).
      const bool padded = (m0 + BM > a.nq) || (n0 + BN > a.ng);
      uint32_t rowok = 0xffffffffu, colok = 0xfu;  // bit i*4+r / bit j: inside the real n_q x n_g
      if (padded) {
        rowok = 0u;
        colok = 0u;
  #pragma unroll
        for (int i = 0; i < TM; ++i)
  #pragma unroll
          for (int r = 0; r < 4; ++r) rowok |= (uint32_t)(rbase + i * 16 + r < a.nq) << (i * 4 + r);
  #pragma unroll
        for (int j = 0; j < TN; ++j) colok |= (uint32_t)(cbase + j * 16 < a.ng) << j;
      }
      uint32_t cc_pack = 0u;  // byte j: count for column j (<= 4*TM per lane, <= 16*TM after the reduce)
      uint32_t und[TM];
      // exact undecided bits of one i-block: lo <= s <= hi from its own compares (reusing
      // "!(s > hi)" kept 128 lane masks live and spilled them); a disabled direction is skipped
      auto und_bits = [&](int i, const f32x4_t& rhi, const f32x4_t& rlo, bool dr, bool dc) {
        uint32_t u = 0u;
  #pragma unroll
        for (int j = 0; j < TN; ++j)
  #pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float sc = acc[i][j][r];
            if (dr) u |= ((sc >= rlo[r] && sc <= rhi[r]) ? 1u : 0u) << (j * 4 + r);
            if (dc) u |= ((sc >= clo[j] && sc <= chi[j]) ? 1u : 0u) << (16 + j * 4 + r);
          }
        return u;
      };
      auto row_reduce = [&](int i, uint32_t rc_pack) {
        // rows: sum over the 16 lanes of a DPP row (those sharing lane >> 4); bytes stay <= 64
        rc_pack = row_sum16(rc_pack);
        if ((lane & 15) == 0) {
  #pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t c = (rc_pack >> (8 * r)) & 0xffu;
            if (c) lds_add_u32_async(&lds_rc[wr * (TM * 16) + i * 16 + (lane >> 4) * 4 + r], (int)c);
          }
        }
      };
      const bool do_row = a.row_hi != nullptr, do_col = a.col_hi != nullptr;
      // scoring pass: per score an exact count compare (v_cmp + v_addc) and the exact "inside [lo, hi]"
      // bit (rank epilogues), or a wave-mask band test with the bits recomputed only where some lane hit
      // (top-k).  The epilogue is VALU-issue-bound (4 cycles per wave64 instruction x 128 scores per
      // lane): every instruction per score counts.
      auto fast_block = [&](auto row_c, auto col_c) {
        constexpr bool DR = decltype(row_c)::value, DC = decltype(col_c)::value;
        uint32_t ccnt[TN] = {};
  #pragma unroll
        for (int i = 0; i < TM; ++i) {
          __builtin_amdgcn_sched_barrier(0);
          f32x4_t rhi = {}, rlo = {};
          if constexpr (DR) {
            rhi = *(const f32x4_t*)(l_rhi + i * 16);
            rlo = *(const f32x4_t*)(l_rlo + i * 16);
          }
          uint32_t c0 = 0u, c1 = 0u, c2 = 0u, c3 = 0u;
          bool hit = false;
          if constexpr (EPI == EPI_TOPK) {
          // top-k emission (a band hit is rare, ~0.1% of scores): a wave-mask hit test, the exact bits
          // recomputed only for i-blocks where some lane hit
  #pragma unroll
          for (int j = 0; j < TN; ++j) {
            const f32x4_t sc = acc[i][j];
            if constexpr (DR) {
              c0 += sc[0] > rhi[0];
              c1 += sc[1] > rhi[1];
              c2 += sc[2] > rhi[2];
              c3 += sc[3] > rhi[3];
  #pragma unroll
              for (int r = 0; r < 4; ++r) hit |= __builtin_amdgcn_fmed3f(sc[r], rlo[r], rhi[r]) == sc[r];
            }
            if constexpr (DC) {
  #pragma unroll
              for (int r = 0; r < 4; ++r) {
                ccnt[j] += sc[r] > chi[j];
                hit |= __builtin_amdgcn_fmed3f(sc[r], clo[j], chi[j]) == sc[r];
              }
            }
          }
          if constexpr (DR) row_reduce(i, c0 | (c1 << 8) | (c2 << 16) | (c3 << 24));
          und[i] = __builtin_amdgcn_ballot_w64(hit) ? und_bits(i, rhi, rlo, DR, DC) : 0u;
          } else {
          // rank counts: the exact count and the exact band bits of every score in one pass -- at the
          // bench data's band rates ~94% of i-blocks hold an undecided pair, so a wave-mask hit test
          // followed by recomputing the bits cost more than writing them directly (16,384 x 131,072 rank
          // pass 3.92 -> 3.83 ms, tools/ab4.sh)
          uint32_t u = 0u;
#ifndef CMVE_EPI_C
#if CMVE_EPI_BOTH_ASM
          if constexpr (DR && DC && TN == 4) {  // both directions (K14 evaluations): hand-scheduled per column block
            uint32_t ur = 0u, uc = 0u;
  #pragma unroll
            for (int j = TN - 1; j >= 0; --j) {  // (bits j * 4 + r, most significant first)
              pair2_count_bits(acc[i][j][3], acc[i][j][2], rhi[3], rlo[3], rhi[2], rlo[2], chi[j], clo[j], c3, c2,
                               ccnt[j], ur, uc);
              pair2_count_bits(acc[i][j][1], acc[i][j][0], rhi[1], rlo[1], rhi[0], rlo[0], chi[j], clo[j], c1, c0,
                               ccnt[j], ur, uc);
            }
            row_reduce(i, c0 | (c1 << 8) | (c2 << 16) | (c3 << 24));
            und[i] = ur | (uc << 16);
            continue;
          }
#endif
#if CMVE_EPI_T2V_DBL
          if constexpr (DR && !DC && TN == 4) {  // t2v (the gallery shape): hand-scheduled per column block
  #pragma unroll
            for (int j = TN - 1; j >= 0; --j)
              col4_count_bits(acc[i][j][3], acc[i][j][2], acc[i][j][1], acc[i][j][0], rhi, rlo, c3, c2, c1, c0, u);
            row_reduce(i, c0 | (c1 << 8) | (c2 << 16) | (c3 << 24));
            und[i] = u;
            continue;
          }
#endif
          if constexpr (DR && !DC && TN == 4) {  // t2v (the bench / gallery shape): hand-scheduled per row
            c0 = row4_count_bits<0>(acc[i][0][0], acc[i][1][0], acc[i][2][0], acc[i][3][0], rhi[0], rlo[0], u);
            c1 = row4_count_bits<1>(acc[i][0][1], acc[i][1][1], acc[i][2][1], acc[i][3][1], rhi[1], rlo[1], u);
            c2 = row4_count_bits<2>(acc[i][0][2], acc[i][1][2], acc[i][2][2], acc[i][3][2], rhi[2], rlo[2], u);
            c3 = row4_count_bits<3>(acc[i][0][3], acc[i][1][3], acc[i][2][3], acc[i][3][3], rhi[3], rlo[3], u);
            row_reduce(i, c0 | (c1 << 8) | (c2 << 16) | (c3 << 24));
            und[i] = u;
            continue;
          }
#endif
  #pragma unroll
          for (int j = 0; j < TN; ++j) {
            const f32x4_t sc = acc[i][j];
            if constexpr (DR) {
              c0 += sc[0] > rhi[0];
              c1 += sc[1] > rhi[1];
              c2 += sc[2] > rhi[2];
              c3 += sc[3] > rhi[3];
  #pragma unroll
              for (int r = 0; r < 4; ++r) u |= (sc[r] >= rlo[r] && sc[r] <= rhi[r]) ? (1u << (j * 4 + r)) : 0u;
            }
            if constexpr (DC) {
  #pragma unroll
              for (int r = 0; r < 4; ++r) {
                ccnt[j] += sc[r] > chi[j];
                u |= (sc[r] >= clo[j] && sc[r] <= chi[j]) ? (1u << (16 + j * 4 + r)) : 0u;
              }
            }
          }
          if constexpr (DR) row_reduce(i, c0 | (c1 << 8) | (c2 << 16) | (c3 << 24));
          und[i] = u;
          }
        }
        if constexpr (DC) {
  #pragma unroll
          for (int j = 0; j < TN; ++j) cc_pack += ccnt[j] << (8 * j);
        }
      };
      if (padded) {  // boundary tiles: out-of-range scores -> -inf (never counted, never in a band)
              for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (!((rowok >> (i * 4 + r)) & (colok >> j) & 1u)) acc[i][j][r] = -INFINITY;
      }
      if (KG > 1 && group != 0) {  // (KG = 2: the second group's sums were added to the first's; it scores nothing)
#pragma unroll
        for (int i = 0; i < TM; ++i) und[i] = 0u;
      } else if (do_row && do_col) {
        fast_block(std::true_type{}, std::true_type{});
      } else if (do_row) {
        fast_block(std::true_type{}, std::false_type{});
      } else {
        fast_block(std::false_type{}, std::true_type{});
      }
      if constexpr (GT_SKIP) {  // drop the GT pairs (row band: column = the row's GT; column band: row = the column's)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          uint32_t m = 0u;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int dc = gt_row[i][r] - cbase;
            m |= (dc >= 0 && dc < TN * 16 && (dc & 15) == 0) ? 1u << ((dc >> 4) * 4 + r) : 0u;
          }
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int dr = gt_col[j] - (rbase + i * 16);
            m |= (dr >= 0 && dr < 4) ? 1u << (16 + j * 4 + dr) : 0u;
          }
          und[i] &= ~m;
        }
      }
      cc_pack += __shfl_xor(cc_pack, 16, 64);
      cc_pack += __shfl_xor(cc_pack, 32, 64);
      if (lane < 16) {
  #pragma unroll
        for (int j = 0; j < TN; ++j) {
          const uint32_t c = (cc_pack >> (8 * j)) & 0xffu;
          if (c) lds_add_u32_async(&lds_cc[wc * (TN * 16) + j * 16 + lane], (int)c);
        }
      }
      CMVE_STAMP(5);
      // emission: exclusive prefix of the per-lane counts, ONE returning global atomic per wave on
      // the tile's bucket counter, issued before the count flush so its latency hides behind the
      // barrier and the flush (a block-wide LDS staging buffer + one atomic per block cost two
      // extra barriers with that atomic's round trip exposed between them: ~40% of the epilogue)
      uint32_t nmine = 0u;
  #pragma unroll
      for (int i = 0; i < TM; ++i) nmine += __builtin_popcount((und[i] | (und[i] >> 16)) & 0xffffu);
      // exclusive prefix of nmine over lanes from one ballot per count bit (mbcnt = popcount of
      // the lower lanes); nmine <= 16*TM < 256.  No LDS round trips (a __shfl scan is 6 bpermutes).
      uint32_t excl = 0u, total = 0u;
      if (__builtin_amdgcn_ballot_w64(nmine != 0u)) {
  #pragma unroll
        for (int b = 0; b < 8; ++b) {
          const unsigned long long m = __builtin_amdgcn_ballot_w64((nmine >> b) & 1u);
          excl += __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << b;
          total += (uint32_t)__builtin_popcountll(m) << b;
        }
      }
      // a tile never straddles buckets (BM, BN <= 256, aligned)
      const int bucket = EPI == EPI_TOPK ? (m0 >> 8)
                                         : (a.tile_buckets ? (m0 >> 6) * a.nbn64 + (n0 >> 6) : (n0 >> CAND_BUCKET_SHIFT));
      unsigned long long wbase = 0ull;
      bool inl = false;  // inline fix-up: the pair total is added after the flush (a returning atomic here stayed
                         // in vmcnt, so the re-score's first load wait also waited for its round trip)
      if constexpr (INL) inl = a.fix_inline != 0;
      if (total && lane == 0 && !inl) wbase = gadd(a.bucket_cnt + bucket, (unsigned long long)total);
      if constexpr (INL) {
        if (a.fix_inline) {
          // fp64 re-score of the tile's undecided pairs (fixup_walk's arithmetic: the same scores), counted
          // into the tile's LDS counts before the flush: the pairs go to an LDS list (wave prefix + this
          // lane's exclusive prefix) and the block's waves take them two at a time, every load of both pairs
          // in flight at once (a pair costs one trip to the raw rows; a 1k-A tile holds ~6)
          if (lane == 0) epi.wtot[wave] = (int)total;
          CMVE_BAR_LDS();
          int woff = 0, ntot = 0;
#pragma unroll
          for (int w = 0; w < NWT; ++w) {
            const int t = epi.wtot[w];
            woff += w < wave ? t : 0;
            ntot += t;
          }
          bool listed = ntot <= CMVE_INL_LIST;
          if (listed && nmine) {
            uint32_t slot = (uint32_t)woff + excl;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
              uint32_t m = (und[i] | (und[i] >> 16)) & 0xffffu;
              while (m) {
                const int bit = __builtin_ctz(m);
                m &= m - 1u;
                const uint32_t lr = (uint32_t)(rbase - m0 + i * 16 + (bit & 3));
                const uint32_t lc = (uint32_t)(cbase - n0 + (bit >> 2) * 16);
                const uint32_t fl = ((und[i] >> bit) & 1u) | (((und[i] >> (16 + bit)) & 1u) << 1);
                epi.list[slot++] = lr | (lc << 8) | (fl << 16);
              }
            }
          }
#ifdef CMVE_DBG_NOINLFIX  // diagnostic build only: no re-score (counts incomplete, results garbage)
          listed = true;
          ntot = 0;
#endif
          if (listed) {
            CMVE_BAR_LDS();
            if (a.q_lo16) {
              // level 2: each wave scores CMVE_L2_P listed pairs at once from the fp16 + bf16 residual planes
              // (l16_scores) and decides every direction whose GT score lies outside s2 +- E2; a pair with a
              // direction left undecided goes to the level-3 list (fp64 in the finish launch, off this kernel's
              // critical path), or -- the list full -- keeps those flags for the fp64 pass below (the wave owns its
              // entries: no other wave touches them)
#if CMVE_L2_PIPE
              // software-pipelined: each wave scores one listed pair per step while the rows of its next pair are
              // already in flight (two pairs' rows in registers, as two pairs per round trip were; the same
              // arithmetic per pair, so the same bits)
              struct L2Stage {
                uint32_t ent;
                int64_t qr, gc;
                float elq, elg;
                L16Frag fq, fg;
              };
              auto l2_fetch = [&](int p, L2Stage& st) {
                st.ent = epi.list[p];
                st.qr = m0 + (st.ent & 0xff);
                st.gc = n0 + ((st.ent >> 8) & 0xff);
                st.elq = gld(a.q_el + st.qr);  // (the row bounds travel with the plane rows)
                st.elg = gld(a.g_el + st.gc);
                const int64_t k = 16 * (int64_t)lane;  // (the level-2 planes need d_pad <= 1024: one chunk)
                if (k < a.ldk) {
                  l16_load(a.qhi + st.qr * a.ldk, a.q_lo16 + st.qr * a.ldk, k, st.fq);
                  l16_load(a.ghi + st.gc * a.ldk, a.g_lo16 + st.gc * a.ldk, k, st.fg);
                }
              };
              auto l2_finish = [&](int p, const L2Stage& st) {
                double s2 = 16 * (int64_t)lane < a.ldk ? l16_partial(st.fq, st.fg, 0.0) : 0.0;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) s2 += __shfl_xor(s2, o, 64);
                if (lane == 0) {
                  const double eq = (double)st.elq, eg = (double)st.elg;
                  const double E2 = eq + (1.0 + eq) * eg + 2e-12;
                  uint32_t fl = (st.ent >> 16) & 3u;
                  const int lr = (int)(st.ent & 0xff), lc = (int)((st.ent >> 8) & 0xff);
                  if (fl & 1u) {
                    const double t = epi.sgt[lr];
                    if (s2 - E2 > t) { lds_add_u32_async(&lds_rc[lr], 1); fl &= ~1u; }
                    else if (s2 + E2 < t) fl &= ~1u;
                  }
                  if (fl & 2u) {
                    const double t = epi.sgt[BM + lc];
                    if (s2 - E2 > t) { lds_add_u32_async(&lds_cc[lc], 1); fl &= ~2u; }
                    else if (s2 + E2 < t) fl &= ~2u;
                  }
                  if (fl && a.l3_count) {  // level 3: counted (a returning atomic: only these few pairs pay it),
                    const unsigned slot = gadd(a.l3_count, 1u);  // listed for the finish (batches) or, with no
                    if (a.l3 && slot < (unsigned)a.l3_cap) {     // list (one evaluation), re-scored right here
                      gst(a.l3 + slot, (unsigned long long)st.qr | ((unsigned long long)st.gc << 31) |
                                           ((unsigned long long)fl << 62));
                      fl = 0u;
                    }
                  }
                  epi.list[p] = (st.ent & 0xffffu) | (fl << 16);
                }
              };
              {
                L2Stage sa, sb;
                int p = wave;
                if (p < ntot) l2_fetch(p, sa);
                while (p < ntot) {  // (two named stages, no register copies)
                  int pn = p + NWT;
                  if (pn < ntot) l2_fetch(pn, sb);
                  l2_finish(p, sa);
                  p = pn;
                  if (p >= ntot) break;
                  pn = p + NWT;
                  if (pn < ntot) l2_fetch(pn, sa);
                  l2_finish(p, sb);
                  p = pn;
                }
              }
#else
              constexpr int RP = BATCH ? ((is_big_ring<BM, BN>() || NW == 4) ? CMVE_L2_P_BIG : CMVE_L2_P) : CMVE_L2_P_ONE;
              for (int p0 = wave * RP; p0 < ntot; p0 += NWT * RP) {
                int64_t qr[RP], gc[RP];
                uint32_t ent[RP];
#pragma unroll
                for (int u = 0; u < RP; ++u) {
                  ent[u] = p0 + u < ntot ? epi.list[p0 + u] : epi.list[p0];  // (a repeat: scored, not used)
                  qr[u] = m0 + (ent[u] & 0xff);
                  gc[u] = n0 + ((ent[u] >> 8) & 0xff);
                }
                // the pairs' row bounds are loaded with their plane rows (as a dependent load after the score
                // they cost the re-score a second round trip)
                float elq[RP], elg[RP];
#pragma unroll
                for (int u = 0; u < RP; ++u) {
                  elq[u] = gld(a.q_el + qr[u]);
                  elg[u] = gld(a.g_el + gc[u]);
                }
                double s2[RP];
                l16_scores<RP>(a, qr, gc, lane, s2);
                if (lane == 0) {
#pragma unroll
                  for (int u = 0; u < RP; ++u) {
                    if (p0 + u >= ntot) break;
                    const double eq = (double)elq[u], eg = (double)elg[u];
                    const double E2 = eq + (1.0 + eq) * eg + 2e-12;
                    uint32_t fl = (ent[u] >> 16) & 3u;
                    const int lr = (int)(ent[u] & 0xff), lc = (int)((ent[u] >> 8) & 0xff);
                    if (fl & 1u) {
                      const double t = epi.sgt[lr];
                      if (s2[u] - E2 > t) { lds_add_u32_async(&lds_rc[lr], 1); fl &= ~1u; }
                      else if (s2[u] + E2 < t) fl &= ~1u;
                    }
                    if (fl & 2u) {
                      const double t = epi.sgt[BM + lc];
                      if (s2[u] - E2 > t) { lds_add_u32_async(&lds_cc[lc], 1); fl &= ~2u; }
                      else if (s2[u] + E2 < t) fl &= ~2u;
                    }
                    if (fl && a.l3_count) {  // level 3: counted (a returning atomic: only these few pairs pay it),
                      const unsigned slot = gadd(a.l3_count, 1u);  // listed for the finish (batches) or, with no
                      if (a.l3 && slot < (unsigned)a.l3_cap) {     // list (one evaluation), re-scored right here
                        gst(a.l3 + slot, (unsigned long long)qr[u] | ((unsigned long long)gc[u] << 31) |
                                             ((unsigned long long)fl << 62));
                        fl = 0u;
                      }
                    }
                    epi.list[p0 + u] = (ent[u] & 0xffffu) | (fl << 16);
                  }
                }
              }
#endif
              CMVE_BAR_LDS();  // the level-2 flags are in LDS for every wave
            }
            auto rescore2 = [&](uint32_t e1, uint32_t e2, bool two) {
              const int64_t r1 = m0 + (e1 & 0xff), c1 = n0 + ((e1 >> 8) & 0xff);
              const int64_t r2 = two ? m0 + (e2 & 0xff) : r1, c2 = two ? n0 + ((e2 >> 8) & 0xff) : c1;
              // the norms travel with the rows (loaded after the dot they were a second round trip)
              const double inv1 = gld(a.q_inv + r1) * gld(a.g_inv + c1), inv2 = gld(a.q_inv + r2) * gld(a.g_inv + c2);
              double d1, d2;
              if (a.q_f64) {
                const double* q = (const double*)a.q_raw;
                if (a.g_f64) {
                  const double* g = (const double*)a.g_raw;
                  wave_dot64_x2(q + r1 * a.q_ld, g + c1 * a.g_ld, q + r2 * a.q_ld, g + c2 * a.g_ld, a.d, lane, d1, d2);
                } else {
                  const float* g = (const float*)a.g_raw;
                  wave_dot64_x2(q + r1 * a.q_ld, g + c1 * a.g_ld, q + r2 * a.q_ld, g + c2 * a.g_ld, a.d, lane, d1, d2);
                }
              } else {
                const float* q = (const float*)a.q_raw;
                if (a.g_f64) {
                  const double* g = (const double*)a.g_raw;
                  wave_dot64_x2(q + r1 * a.q_ld, g + c1 * a.g_ld, q + r2 * a.q_ld, g + c2 * a.g_ld, a.d, lane, d1, d2);
                } else {
                  const float* g = (const float*)a.g_raw;
                  wave_dot64_x2(q + r1 * a.q_ld, g + c1 * a.g_ld, q + r2 * a.q_ld, g + c2 * a.g_ld, a.d, lane, d1, d2);
                }
              }
              if (lane == 0) {
                const double s1 = d1 * inv1;  // wave_cos64
                if ((e1 >> 16) & 1u) { if (s1 > epi.sgt[r1 - m0]) lds_add_u32_async(&lds_rc[r1 - m0], 1); }
                if ((e1 >> 17) & 1u) { if (s1 > epi.sgt[BM + c1 - n0]) lds_add_u32_async(&lds_cc[c1 - n0], 1); }
                if (two) {
                  const double s2 = d2 * inv2;
                  if ((e2 >> 16) & 1u) { if (s2 > epi.sgt[r2 - m0]) lds_add_u32_async(&lds_rc[r2 - m0], 1); }
                  if ((e2 >> 17) & 1u) { if (s2 > epi.sgt[BM + c2 - n0]) lds_add_u32_async(&lds_cc[c2 - n0], 1); }
                }
              }
            };
            // batches: one pair per wave at a time (64 registers of rows in flight, not 128), so that the kernel's
            // register count leaves room on each SIMD for a wave of the other stream's prep
            constexpr bool FIX1 = BATCH && CMVE_BATCH_FIX1;
            if constexpr (FIX1) {
              for (int p = wave; p < ntot; p += NWT) {
                const uint32_t e = epi.list[p];
                if (!(e >> 16)) continue;  // decided at level 2
                const int64_t r1 = m0 + (e & 0xff), c1 = n0 + ((e >> 8) & 0xff);
                const double inva = gld(a.q_inv + r1), invb = gld(a.g_inv + c1);
                double s1;
                if (a.q_f64) {
                  const double* x = (const double*)a.q_raw + r1 * a.q_ld;
                  s1 = a.g_f64 ? wave_cos64(x, (const double*)a.g_raw + c1 * a.g_ld, inva, invb, a.d, lane)
                               : wave_cos64(x, (const float*)a.g_raw + c1 * a.g_ld, inva, invb, a.d, lane);
                } else {
                  const float* x = (const float*)a.q_raw + r1 * a.q_ld;
                  s1 = a.g_f64 ? wave_cos64(x, (const double*)a.g_raw + c1 * a.g_ld, inva, invb, a.d, lane)
                               : wave_cos64(x, (const float*)a.g_raw + c1 * a.g_ld, inva, invb, a.d, lane);
                }
                if (lane == 0) {
                  if ((e >> 16) & 1u) { if (s1 > epi.sgt[r1 - m0]) lds_add_u32_async(&lds_rc[r1 - m0], 1); }
                  if ((e >> 17) & 1u) { if (s1 > epi.sgt[BM + c1 - n0]) lds_add_u32_async(&lds_cc[c1 - n0], 1); }
                }
              }
            } else if (a.q_lo16) {  // level 3 after level 2 (a full level-3 list): one pair at a time per wave
              for (int p = wave; p < ntot; p += NWT) {
                const uint32_t e = epi.list[p];
                if (e >> 16) rescore2(e, 0u, false);
              }
            } else {
              for (int p = 2 * wave; p < ntot; p += 2 * NWT)
                rescore2(epi.list[p], p + 1 < ntot ? epi.list[p + 1] : 0u, p + 1 < ntot);
            }
          } else {
            // more than the list holds (a pathological tile): each wave re-scores its own pairs in turn
#pragma unroll
            for (int i = 0; i < TM; ++i) {
              uint32_t bits = (und[i] | (und[i] >> 16)) & 0xffffu;
              unsigned long long m;
              while ((m = __builtin_amdgcn_ballot_w64(bits != 0u))) {
                const int src = (int)__builtin_ctzll(m);
                const uint32_t sb = (uint32_t)__builtin_amdgcn_readlane((int)bits, src);
                const uint32_t su = (uint32_t)__builtin_amdgcn_readlane((int)und[i], src);
                const int bit = __builtin_ctz(sb);
                if (lane == src) bits &= bits - 1u;
                const int lr = wr * (TM * 16) + (src >> 4) * 4 + i * 16 + (bit & 3);
                const int lc = wc * (TN * 16) + (src & 15) + (bit >> 2) * 16;
                const int64_t row = m0 + lr, col = n0 + lc;
                const double inva = gld(a.q_inv + row), invb = gld(a.g_inv + col);
                double sc;
                if (a.q_f64) {
                  const double* x = (const double*)a.q_raw + row * a.q_ld;
                  sc = a.g_f64 ? wave_cos64(x, (const double*)a.g_raw + col * a.g_ld, inva, invb, a.d, lane)
                               : wave_cos64(x, (const float*)a.g_raw + col * a.g_ld, inva, invb, a.d, lane);
                } else {
                  const float* x = (const float*)a.q_raw + row * a.q_ld;
                  sc = a.g_f64 ? wave_cos64(x, (const double*)a.g_raw + col * a.g_ld, inva, invb, a.d, lane)
                               : wave_cos64(x, (const float*)a.g_raw + col * a.g_ld, inva, invb, a.d, lane);
                }
                if (lane == 0) {
                  if (((su >> bit) & 1u) && sc > epi.sgt[lr]) lds_add_u32_async(&lds_rc[lr], 1);
                  if (((su >> (16 + bit)) & 1u) && sc > epi.sgt[BM + lc]) lds_add_u32_async(&lds_cc[lc], 1);
                }
              }
            }
          }
        }
      }
      CMVE_STAMP(6);
#ifdef CMVE_DBG_NOFLUSH  // diagnostic build only: no global flush of candidates / counts (results garbage)
      for (int t = tid; t < BM + BN; t += NTT) lds_rc[t] = 0;
      return;
#endif
      CMVE_BAR_LDS();  // every wave's row / column count adds have landed in LDS
      for (int t = tid; t < BM + BN; t += NTT) {
        const int c = lds_rc[t];
        lds_rc[t] = 0;  // owner thread: ready for the next tile
        if (!c) continue;
        if (t < BM) {
          if (a.row_cnt && m0 + t < a.nq) gadd(a.row_cnt + m0 + t, c);
        } else {
          if (a.col_cnt && n0 + t - BM < a.ng) gadd(a.col_cnt + n0 + t - BM, c);
        }
      }
      if (inl && total && lane == 0) gadd(a.bucket_cnt + bucket, (unsigned long long)total);  // (no return)
      const bool emit = total != 0u && !inl;  // (inline: re-scored above; the bucket count is the pair total)
      if (emit) {
        const unsigned long long w0 = __shfl(wbase, 0, 64);  // this wave's first slot in the bucket
        // K14 with a fix-up launch (SimArgs::ovf_inline): a wave whose pairs do not all fit its bucket re-scores
        // them here in fp64 (into the global counts, after the flush) and leaves null entries in the slots it
        // reserved -- an evaluation never overflows (tiles dense with undecided pairs: near-duplicate rows)
        bool rescue = false;
        if constexpr (INL) rescue = a.ovf_inline && w0 + total > (unsigned long long)a.cap_b;
        unsigned long long slot = w0 + excl;
        unsigned long long* dst = a.cand + (size_t)bucket * a.cap_b;
  #pragma unroll
        for (int i = 0; i < TM; ++i) {
          uint32_t m = (und[i] | (und[i] >> 16)) & 0xffffu;
          while (m) {
            const int bit = __builtin_ctz(m);
            m &= m - 1u;
            unsigned long long packed;
            if constexpr (EPI == EPI_TOPK) {
              // key(s) << 32 | (row & 255) << 24 | col: the bucket (m0 >> 8) holds the row's high bits
              float sc = acc[i][0][0];
  #pragma unroll
              for (int jj = 0; jj < TN; ++jj)
  #pragma unroll
                for (int r = 0; r < 4; ++r) sc = (bit == jj * 4 + r) ? acc[i][jj][r] : sc;
              packed = ((unsigned long long)topk_key(sc) << 32) |
                       ((unsigned long long)((rbase + i * 16 + (bit & 3)) & 255) << 24) |
                       (unsigned long long)(cbase + (bit >> 2) * 16);
            } else {
              const unsigned long long flags = ((und[i] >> bit) & 1u) | (((und[i] >> (16 + bit)) & 1u) << 1);
              packed = rescue ? 0ull
                              : (unsigned long long)(rbase + i * 16 + (bit & 3)) |
                                    ((unsigned long long)(cbase + (bit >> 2) * 16) << 31) | (flags << 62);
            }
            if ((long long)slot < a.cap_b) gst(dst + slot, packed);
            ++slot;
          }
        }
        if constexpr (INL) {
          if (rescue) {  // (wave-uniform) the wave's pairs one at a time: fixup_walk's arithmetic, global counts
#pragma unroll
            for (int i = 0; i < TM; ++i) {
              uint32_t bits = (und[i] | (und[i] >> 16)) & 0xffffu;
              unsigned long long mm;
              while ((mm = __builtin_amdgcn_ballot_w64(bits != 0u))) {
                const int src = (int)__builtin_ctzll(mm);
                const uint32_t sb = (uint32_t)__builtin_amdgcn_readlane((int)bits, src);
                const uint32_t su = (uint32_t)__builtin_amdgcn_readlane((int)und[i], src);
                const int bit = __builtin_ctz(sb);
                if (lane == src) bits &= bits - 1u;
                const int64_t row = m0 + wr * (TM * 16) + (src >> 4) * 4 + i * 16 + (bit & 3);
                const int64_t col = n0 + wc * (TN * 16) + (src & 15) + (bit >> 2) * 16;
                const double inva = gld(a.q_inv + row), invb = gld(a.g_inv + col);
                double sc;
                if (a.q_f64) {
                  const double* x = (const double*)a.q_raw + row * a.q_ld;
                  sc = a.g_f64 ? wave_cos64(x, (const double*)a.g_raw + col * a.g_ld, inva, invb, a.d, lane)
                               : wave_cos64(x, (const float*)a.g_raw + col * a.g_ld, inva, invb, a.d, lane);
                } else {
                  const float* x = (const float*)a.q_raw + row * a.q_ld;
                  sc = a.g_f64 ? wave_cos64(x, (const double*)a.g_raw + col * a.g_ld, inva, invb, a.d, lane)
                               : wave_cos64(x, (const float*)a.g_raw + col * a.g_ld, inva, invb, a.d, lane);
                }
                if (lane == 0) {
                  if (((su >> bit) & 1u) && sc > gld(a.row_sgt + row)) gadd(a.row_cnt + row, 1);
                  if (((su >> (16 + bit)) & 1u) && sc > gld(a.col_sgt + col)) gadd(a.col_cnt + col, 1);
                }
              }
            }
          }
        }
      }
  #ifdef CMVE_DBG_STAMPS
      CMVE_BAR_LDS();
  #endif
      CMVE_STAMP(3);
    }
  };

  const int frow = lane & 15;
  if constexpr (PHASED) {
    // ---- G256 phased schedule (2 buffers of BK=64, 4 phases per K-tile, 2 staggered groups) ----
    // phase = { ds_read subtile, [LDS-DMA issue], [counted vmcnt], s_barrier,
    //           16 MFMAs (one 64x32 quadrant of the wave's 128x64 tile, K=64), s_barrier }.
    // Group 1 (waves 4-7, wr = 1) runs one barrier behind group 0, so on every SIMD (waves w and
    // w+4) one wave issues MFMAs while the other reads LDS / issues loads.
    //   K-tile t (buffer t&1):   r=1 reads A(qm0)+B(qn0), MFMA Q00;  r=2 reads B(qn1), Q01;
    //                            r=3 reads A(qm1), Q11;               r=4 no reads, Q10.
    //   loads: A(t+1) at r=1 (its buffer's A was last read 2 phases earlier, r=3 of t-1),
    //          B(t+2) at r=4 (this buffer's B was last read at r=2); r=4 waits for K-tile t+1
    //          with only B(t+2) younger: vmcnt(4) -- 3 to 4 phases for every load to land.
    // RAW: a wait before phase p's first barrier covers reads from phase p+1 on, for both groups;
    // WAR: a buffer is restaged >= 2 phases after its last ds_read (cdna_hip_programming.md Sec.5).
    static_assert(BM == 256 && BN == 256 && TM == 8 && TN == 4 && NW == 8, "phased path is the 256x256 geometry");
    const int ldk_b = (int)(a.ldk * 2);
    auto rsrc_of = [&](const uint16_t* base, int row0, int rows) {
      return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (int64_t)row0 * a.ldk), 0, rows * ldk_b, 0x00020000);
    };
    __amdgpu_buffer_rsrc_t rA = rsrc_of(a.qhi, m0, BM);
    __amdgpu_buffer_rsrc_t rB = rsrc_of(a.ghi, n0, BN);
    // split-bf16: the lo planes too (plane_of picks per K-tile); else unused copies
    __amdgpu_buffer_rsrc_t rAl = rA, rBl = rB;
    if constexpr (MODE == CMVE_SIM_BF16X3) {
      rAl = rsrc_of(a.qlo, m0, BM);
      rBl = rsrc_of(a.glo, n0, BN);
    }
    // piece = 8 rows x 128 B (one wave-instruction, 1 KiB): lane l -> row l>>3, LDS chunk l&7,
    // global chunk (l&7) ^ (row&7)
    const int voff = (lane >> 3) * ldk_b + (((lane & 7) ^ (lane >> 3)) << 4);
    auto stage_op = [&](const __amdgpu_buffer_rsrc_t& rhi, int t, int plane_off) {
#ifdef CMVE_DBG_NOLOAD  // diagnostic build only: MFMA + LDS-read ceiling (results are garbage)
      return;
#endif
      char* dst = smem + (t & 1) * STAGE_BYTES + plane_off;
      bool alo = false, blo = false;
      int kt = t;
      if constexpr (MODE == CMVE_SIM_BF16X3) plane_of(t, alo, blo, kt);
      const bool lo_plane = plane_off == 0 ? alo : blo;
      const __amdgpu_buffer_rsrc_t r = !lo_plane ? rhi : (plane_off == 0 ? rAl : rBl);
      const int kb = kt * (BK * 2);
#pragma unroll
      for (int it = 0; it < 4; ++it) {  // 32 pieces per 256-row plane, 4 per wave
        const int piece = wave * 4 + it;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(dst + piece * 1024), 16, voff,
                                                 piece * 8 * ldk_b + kb, 0, 0);
      }
    };
    const int nk = a.nk;
    // fragment address: row (tile row + frow), chunk (ks*4 + lane>>4) ^ (row & 7) with row&7 == lane&7
    const int c0 = ((0 + (lane >> 4)) ^ (lane & 7)) << 4, c1 = ((4 + (lane >> 4)) ^ (lane & 7)) << 4;
    const int arow = (wr * 128 + frow) * 128, brow = A_BYTES + (wc * 64 + frow) * 128;
    s16x8_t fa[4][2], fb0[2][2], fb1[2][2];
    auto read_a = [&](const char* buf, int qm) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const char* p = buf + arow + (qm * 64 + i * 16) * 128;
        fa[i][0] = *(const s16x8_t*)(p + c0);
        fa[i][1] = *(const s16x8_t*)(p + c1);
      }
    };
    auto read_b = [&](const char* buf, int qn, s16x8_t (&fb)[2][2]) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const char* p = buf + brow + (qn * 32 + j * 16) * 128;
        fb[j][0] = *(const s16x8_t*)(p + c0);
        fb[j][1] = *(const s16x8_t*)(p + c1);
      }
    };
    auto quadrant = [&](int qm, int qn, const s16x8_t (&fb)[2][2]) {
#ifdef CMVE_DBG_NOMFMA  // diagnostic build only: staging + LDS-read floor (results are garbage)
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(fa[i][0]), "v"(fa[i][1]));
#pragma unroll
      for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(fb[j][0]), "v"(fb[j][1]));
#else
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[qm * 4 + i][qn * 2 + j] = mfma<MODE>(fa[i][ks], fb[j][ks], acc[qm * 4 + i][qn * 2 + j]);
      __builtin_amdgcn_s_setprio(0);
#endif
    };
#define CMVE_BAR()                                  \
  __builtin_amdgcn_sched_barrier(0);                \
  asm volatile("s_barrier" ::: "memory");           \
  __builtin_amdgcn_sched_barrier(0)

    // a tile's first loads: K-tile 0 (A, B) and B(1).  For every tile after a block's first they
    // are issued before the previous tile's epilogue, whose ~10k cycles hide their latency.
    auto prologue_loads = [&]() {
      stage_op(rA, 0, 0);
      stage_op(rB, 0, A_BYTES);
      if (nk > 1) stage_op(rB, 1, A_BYTES);
    };
    prologue_loads();
    for (;;) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    CMVE_BAR();
    CMVE_STAMP(1);
    if (wr == 1) { CMVE_BAR(); }  // stagger: group 1 runs one barrier behind
    for (int t = 0; t < nk; ++t) {
      const char* buf = smem + (t & 1) * STAGE_BYTES;
      // r = 1
      if (t + 1 < nk) stage_op(rA, t + 1, 0);
      read_a(buf, 0);
      read_b(buf, 0, fb0);
      CMVE_BAR();
      quadrant(0, 0, fb0);
      CMVE_BAR();
      // r = 2
      read_b(buf, 1, fb1);
      CMVE_BAR();
      quadrant(0, 1, fb1);
      CMVE_BAR();
      // r = 3
      read_a(buf, 1);
      CMVE_BAR();
      quadrant(1, 1, fb1);
      CMVE_BAR();
      // r = 4: restage B of this buffer with K-tile t+2; K-tile t+1 must have landed
      if (t + 2 < nk) {
        stage_op(rB, t + 2, A_BYTES);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      CMVE_BAR();
      quadrant(1, 0, fb0);
      CMVE_BAR();
    }
    if (wr == 0) { CMVE_BAR(); }  // re-align the barrier counts of the two groups
    CMVE_STAMP(2);
    // every K-tile of this tile has been read (both groups passed the realigning barrier): the
    // staging buffers are free for the next tile while this one's epilogue runs
    const int next = tile + (int)gridDim.x;
    const bool has_next = next < ntiles;
    int m0n = 0, n0n = 0;
    float thn_hi = 0.f, thn_lo = 0.f;
    float coln[NCV][TN];
    if (has_next) {
      tile_origin(next, m0n, n0n);
      rA = rsrc_of(a.qhi, m0n, BM);
      rB = rsrc_of(a.ghi, n0n, BN);
      if constexpr (MODE == CMVE_SIM_BF16X3) {
        rAl = rsrc_of(a.qlo, m0n, BM);
        rBl = rsrc_of(a.glo, n0n, BN);
      }
      prologue_loads();
      if constexpr (epi_thr(EPI)) fetch_thr(m0n, n0n, thn_hi, thn_lo);
      if constexpr (EPI_COLS) fetch_cols(n0n, coln);
    }
    epilogue();
    if (!has_next) break;
    if constexpr (EPI_COLS)
#pragma unroll
      for (int c = 0; c < NCV; ++c)
#pragma unroll
        for (int j = 0; j < TN; ++j) colv[c][j] = coln[c][j];
    tile = next;
    m0 = m0n;
    n0 = n0n;
    thr_hi_v = thn_hi;
    thr_lo_v = thn_lo;
    for (int i = 0; i < TM; ++i)
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
#undef CMVE_BAR
  } else if constexpr (RING) {
  // ---- ring of NS stages (G64): K-tiles t+1 .. t+NS-2 stay in flight while K-tile t is consumed ----
  constexpr int RPI = 64 / (KB / 8);  // rows per staging wave-instruction (1 KiB)
  constexpr int LPS = (BM / RPI / NW + BN / RPI / NW) * (MODE == CMVE_SIM_BF16X3 ? 2 : 1);  // loads / stage / wave
  constexpr int KS = KB / 32;  // 32-deep MFMA steps per K-tile
#ifndef CMVE_RING_KSPLIT
#define CMVE_RING_KSPLIT 0
#endif
  // the batch rings with CMVE_RING_KSPLIT: fragments and MFMAs one 32-deep step at a time
  constexpr bool KSPLIT = CMVE_RING_KSPLIT && BATCH && MODE != CMVE_SIM_BF16X3 && KS > 1;
  static_assert(LPS * (NS - 2) <= 63, "vmcnt immediate");
  const int nk0 = a.nk0 * (BK / KB);  // (a.nk0: 64-deep K-tiles; d_pad % 64 == 0)
  // KG = 2: this wave's group streams K-tiles [kt0, kt0 + nkg) (the host launches it only for nk0 % 2 == 0)
  const int nkg = nk0 / KG, kt0 = group * nkg;
  // the K-tile streamed at step t: in order, or (CMVE_RING_KROT study) rotated per tile, so the tiles of an XCD that
  // run in lockstep read different K-slices of their shared panels at any moment (each tile's own sum in another
  // order: the scores move within the error bound, the ranks do not)
#if CMVE_RING_KROT
  const int krot = BATCH ? (int)(((unsigned)(m0 / BM) * 3u + (unsigned)(n0 / BN) * 5u) % (unsigned)max(nkg, 1)) : 0;
  auto kt_of = [&](int t) { const int u = t + krot; return kt0 + (u >= nkg ? u - nkg : u); };
#else
  auto kt_of = [&](int t) { return kt0 + t; };
#endif
  // K14: the other set's err_max shards as VECTOR loads, one shard per lane, issued before the first
  // K-tiles (the oldest loads: retired by the first ring wait) and folded after the main loop -- as scalar
  // loads their round trip held the prologue (~2.5 us to the first K-tile in the stamps)
  static_assert(EVAL_EMAX_SHARDS == 64, "one err_max shard per lane");
  unsigned emq = 0u, emg = 0u;
  if constexpr (epi_thr(EPI)) {
    if (a.thr_gt) {
      emq = gld(a.q_emax + lane);
      emg = gld(a.g_emax + lane);
    }
  }
  // CMVE_RING_VGPR_STAGE (the batch ring): K-tiles staged through registers -- global_load_dwordx4 of the same 16 B per
  // lane an LDS-DMA piece moves, ds_write_b128 into the same LDS image -- one K-tile ahead in registers, one in LDS
  // (an LDS-DMA piece costs its wave ~100-185 issue cycles inside a phase of MFMAs and fragment reads,
  // MI355X_MICROARCH.md: 8 per wave per K-tile, the main loop's largest single cost)
  constexpr bool RSTG = CMVE_RING_VGPR_STAGE && BATCH && MODE != CMVE_SIM_BF16X3 && KG == 1 && NS == 2;
  constexpr int PWA = RSTG ? BM / RPI / NW : 1, PWB = RSTG ? BN / RPI / NW : 1;
  cmve_u32x4 stg_a[PWA], stg_b[PWB];
  auto rload = [&](int t) {
    const int k0 = t * KB;
    const char* ba = (const char*)(st_qhi + ((int64_t)m0 + lw * PWA * RPI) * st_ldk + k0);
    const char* bb = (const char*)(st_ghi + ((int64_t)n0 + lw * PWB * RPI) * st_ldk + k0);
#pragma unroll
    for (int it = 0; it < PWA; ++it) stg_a[it] = gld((const cmve_u32x4*)(ba + (int64_t)it * RPI * st_ldk * 2 + st_loff));
#pragma unroll
    for (int it = 0; it < PWB; ++it) stg_b[it] = gld((const cmve_u32x4*)(bb + (int64_t)it * RPI * st_ldk * 2 + st_loff));
  };
  auto rstore = [&](int s) {
    char* base = smem + s * STAGE_BYTES;
#pragma unroll
    for (int it = 0; it < PWA; ++it) *(cmve_u32x4*)(base + (lw * PWA + it) * 1024 + lane * 16) = stg_a[it];
#pragma unroll
    for (int it = 0; it < PWB; ++it) *(cmve_u32x4*)(base + A_BYTES + (lw * PWB + it) * 1024 + lane * 16) = stg_b[it];
  };
  if constexpr (RSTG) {
    if (nkg > 0) {
      rload(kt0);
      rstore(0);
    }
    if (nkg > 1) rload(kt0 + 1);
  } else {
    for (int t = 0; t < NS - 1 && t < nkg; ++t) stage(kt_of(t), t);
  }
  // K14 thresholds: the GT score / bound loads are issued behind the first K-tiles' loads and the rule
  // applied after the main loop (using them at once would wait vmcnt(0), i.e. for every staged K-tile)
  double sgt_raw = 0.0;
  float e_raw = 0.f;
  const bool thr_dir = tid < BM ? a.row_hi != nullptr : (tid < BM + BN && a.col_hi != nullptr);
  if constexpr (epi_thr(EPI)) {
    if (a.thr_gt) {
      if (thr_dir) {
        sgt_raw = tid < BM ? gld(a.row_sgt + m0 + tid) : gld(a.col_sgt + n0 + tid - BM);
        e_raw = tid < BM ? gld(a.q_err + m0 + tid) : gld(a.g_err + n0 + tid - BM);
      }
      fetch_gt1();
    }
  }
  CMVE_STAMP(1);
#ifdef CMVE_STUDY_LOOP_PRIO  // study: the batch ring's main loop at a raised wave priority (the co-resident preps' waves
  if constexpr (BATCH) __builtin_amdgcn_s_setprio(CMVE_STUDY_LOOP_PRIO);  // stay at 0)
#endif
  for (int t = 0; t < nkg; ++t) {
    // K-tile t has landed once at most LPS * (newer stages in flight) loads of this wave are outstanding
    const int newer = RSTG ? -1 : min(NS - 2, nkg - 1 - t);  // (RSTG: K-tile t is in LDS, its loads long waited for)
    switch (newer) {
      case -1: break;
#define CMVE_RING_WAIT(k) \
  case k: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS * (k)) : "memory"); break;
      CMVE_RING_WAIT(0) CMVE_RING_WAIT(1) CMVE_RING_WAIT(2) CMVE_RING_WAIT(3) CMVE_RING_WAIT(4) CMVE_RING_WAIT(5)
      CMVE_RING_WAIT(6)
#undef CMVE_RING_WAIT
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // every wave's share of K-tile t is in LDS, every wave is done with K-tile t-1 (an LDS-only barrier:
    // __syncthreads would drain vmcnt, i.e. the ring)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#if CMVE_RING_READS_FIRST
    // the same drain as a builtin the compiler's wait-count pass sees: with a scalar load it believes outstanding
    // (the asm above is opaque to it) every LDS-read wait below would be lgkmcnt(0) instead of counted
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt / expcnt left at their maxima (gfx9 encoding)
#endif
    if constexpr (!RSTG)
      if (t + NS - 1 < nkg) stage(kt_of(t + NS - 1), (t + NS - 1) % NS);  // refills K-tile t-1's buffer
    const char* base = smem + (group * NS + t % NS) * STAGE_BYTES;
    const char* pA = base;
    const char* pB = base + A_BYTES;
    if constexpr (KSPLIT) {
      // one 32-deep step at a time: its fragments, then its MFMAs (half the fragment registers live)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int chunk = ks * 4 + (lane >> 4);
        s16x8_t fa1[TM], fb1[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) fb1[j] = read_frag<KB>(pB, wc * (TN * 16) + j * 16 + frow, chunk);
#pragma unroll
        for (int i = 0; i < TM; ++i) fa1[i] = read_frag<KB>(pA, wr * (TM * 16) + i * 16 + frow, chunk);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma<MODE>(fa1[i], fb1[j], acc[i][j]);
      }
      continue;
    }
    s16x8_t fa[KS][TM], fb[KS][TN];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int chunk = ks * 4 + (lane >> 4);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[ks][j] = read_frag<KB>(pB, wc * (TN * 16) + j * 16 + frow, chunk);
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[ks][i] = read_frag<KB>(pA, wr * (TM * 16) + i * 16 + frow, chunk);
    }
#if CMVE_RING_READS_FIRST
    // every fragment read of the K-tile issued before its first MFMA: each 32-deep step's MFMAs wait (counted
    // lgkmcnt) only for their own reads, the later step's reads land under the earlier step's MFMAs (left to the
    // scheduler, the reads went out in groups of 6 and 2, each drained by lgkmcnt(0) right before its MFMAs)
    __builtin_amdgcn_sched_barrier(0);
#endif
    if constexpr (MODE == CMVE_SIM_BF16X3) {  // pairs (lo, hi) then (hi, lo): plane_of's order
      const char* pAl = base + A_BYTES + B_BYTES;
      const char* pBl = base + 2 * A_BYTES + B_BYTES;
      s16x8_t lx[KS][TM > TN ? TM : TN];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int chunk = ks * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < TM; ++i) lx[ks][i] = read_frag<KB>(pAl, wr * (TM * 16) + i * 16 + frow, chunk);
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma<MODE>(lx[ks][i], fb[ks][j], acc[i][j]);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int chunk = ks * 4 + (lane >> 4);
#pragma unroll
        for (int j = 0; j < TN; ++j) lx[ks][j] = read_frag<KB>(pBl, wc * (TN * 16) + j * 16 + frow, chunk);
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma<MODE>(fa[ks][i], lx[ks][j], acc[i][j]);
    }
#ifdef CMVE_DBG_NOMFMA  // diagnostic build only: the fragments are read, no MFMA issued (results garbage)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(fa[ks][i]));
#pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(fb[ks][j]));
    }
#else
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma<MODE>(fa[ks][i], fb[ks][j], acc[i][j]);
#endif
    if constexpr (RSTG) {  // K-tile t+1 into the other buffer (read by every wave before the barrier above), t+2 loaded
      if (t + 1 < nkg) {
        rstore((t + 1) % NS);
        if (t + 2 < nkg) rload(kt0 + t + 2);
      }
    }
  }
#ifdef CMVE_STUDY_LOOP_PRIO
  if constexpr (BATCH) __builtin_amdgcn_s_setprio(0);
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the threshold loads, if any are still out)
  if constexpr (epi_thr(EPI)) {
    if (a.thr_gt) {  // fold the shards: a wave max (every lane the same bits)
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        emq = max(emq, (unsigned)__shfl_xor((int)emq, o, 64));
        emg = max(emg, (unsigned)__shfl_xor((int)emg, o, 64));
      }
      qmax_v = __uint_as_float(emq);
      gmax_v = __uint_as_float(emg);
    }
    if (a.thr_gt && thr_dir) thr_of(sgt_raw, e_raw, tid < BM ? gmax_v : qmax_v, thr_hi_v, thr_lo_v);
    if constexpr (INL) sgt_pub = sgt_raw;  // (after the main loop: the load has been waited for)
  }
  if constexpr (KG > 1) {
    // the second group's partial sums into the first's, through the second group's own (now idle) ring: a barrier
    // (every wave done reading its ring), group 1 stores, a barrier, group 0 adds; group 1's accumulators become
    // -inf, which no threshold counts and no band holds (it skips the scoring anyway)
    static_assert(KG == 2 && NS * STAGE_BYTES >= NT * TM * TN * 16, "the partials fit the second group's ring");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    f32x4_t* part = (f32x4_t*)(smem + NS * STAGE_BYTES) + (size_t)(lw * 64 + lane) * (TM * TN);
    if (group == 1) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) part[i * TN + j] = acc[i][j];
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (group == 0) {
          acc[i][j] += part[i * TN + j];
        } else {
          acc[i][j] = f32x4_t{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
        }
      }
  }
  CMVE_STAMP(2);
  } else {
  stage(0, 0);
  if constexpr (epi_thr(EPI)) {
    if (a.thr_gt) {  // overlaps the first K-tile's loads
      reduce_err_max();
      fetch_thr(m0, n0, thr_hi_v, thr_lo_v);
      fetch_gt1();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int t = 0; t < a.nk0; ++t) {
    if (t + 1 < a.nk0) stage(t + 1, (t + 1) & 1);
    const char* base = smem + (t & 1) * STAGE_BYTES;
    const char* pA = base;
    const char* pB = base + A_BYTES;
    // all fragments of this K step first (the compiler's counted lgkmcnt waits let the first
    // MFMAs start on the first fragments), then ONE MFMA cluster: no LDS round trip inside it
    s16x8_t fa[2][TM], fb[2][TN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = ks * 4 + (lane >> 4);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[ks][j] = read_frag(pB, wc * (TN * 16) + j * 16 + frow, chunk);
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[ks][i] = read_frag(pA, wr * (TM * 16) + i * 16 + frow, chunk);
    }
    __builtin_amdgcn_sched_barrier(0);
#ifdef CMVE_DBG_NOMFMA
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(fa[ks][i]));
#pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(fb[ks][j]));
    }
#else
    if constexpr (MODE == CMVE_SIM_BF16X3) {  // pairs (lo, hi) then (hi, lo): plane_of's order
      const char* pAl = base + A_BYTES + B_BYTES;
      const char* pBl = base + 2 * A_BYTES + B_BYTES;
      s16x8_t lx[2][TM > TN ? TM : TN];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int chunk = ks * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < TM; ++i) lx[ks][i] = read_frag(pAl, wr * (TM * 16) + i * 16 + frow, chunk);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma<MODE>(lx[ks][i], fb[ks][j], acc[i][j]);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int chunk = ks * 4 + (lane >> 4);
#pragma unroll
        for (int j = 0; j < TN; ++j) lx[ks][j] = read_frag(pBl, wc * (TN * 16) + j * 16 + frow, chunk);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma<MODE>(fa[ks][i], lx[ks][j], acc[i][j]);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma<MODE>(fa[ks][i], fb[ks][j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  }

  if constexpr (!PHASED) epilogue();
}

// the launch geometry's fields of SimArgs: tile grid and the tile-order group width
static void geo_fill(SimArgs& a, int64_t nq_pad, int64_t ng_pad, int bm, int bn) {
  a.nblk_m = (int)(nq_pad / bm);
  a.nblk_n = (int)(ng_pad / bn);
  a.gn = CMVE_SIM_GN;
}

template <int MODE, int EPI, int WM, int WN, int TM, bool PHASED, int KG = 1>
static int launch_geo(SimArgs a, int64_t nq_pad, int64_t ng_pad, hipStream_t stream) {
  using G = Geo<WM, WN, TM>;
  // + the static epilogue scratch (EpiLds); KG = 2: a ring per K group
  const size_t lds = ring_lds_bytes<MODE, G::BM, G::BN, PHASED, G::NW>() * KG;
  // once per instantiation; function-local static init is thread-safe (one host thread per shard / GPU)
  static const hipError_t attr_err = hipFuncSetAttribute(
      (const void*)sim_kernel<MODE, EPI, WM, WN, TM, PHASED, false, KG>, hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)lds);
  CMVE_HIP(attr_err);
  geo_fill(a, nq_pad, ng_pad, G::BM, G::BN);
  unsigned nblocks = (unsigned)a.nblk_m * (unsigned)a.nblk_n;
  if constexpr (PHASED) {  // persistent: one block per CU (a multiple of 8: the XCD map is blockIdx & 7)
    const int cus = std::max(8, device_cus() / 8 * 8);
    nblocks = std::min<unsigned>(nblocks, (unsigned)cus);
  }
  cmve::launch(sim_kernel<MODE, EPI, WM, WN, TM, PHASED, false, KG>, dim3(nblocks), dim3(G::NT * KG), (uint32_t)lds,
               stream, a, (const SimArgs*)nullptr);
  return check_launch("sim_kernel");
}

// G256 (phased schedule) for bf16/fp16 when both sides tile by 256 and the grid has >= 512
// tiles; G64 below 128 tiles of 128^2; else G128 (2-stage).  Study builds (make study DEFS=-DCMVE_SIM_GEO=128 / 2562)
// force G128 / the 2-stage G256 loop; the product build reads no environment.
static constexpr int sim_geo_force() { return CMVE_SIM_GEO; }

// true when launch_sim takes the persistent phased G256 kernel (which reads explicit thresholds only)
static bool sim_uses_phased(int mode, int64_t nq_pad, int64_t ng_pad) {
  const int force = sim_geo_force();
  if (force == 128 || nq_pad % 256 || ng_pad % 256 || (nq_pad / 256) * (ng_pad / 256) < 512) return false;
  return !(force == 2562 && mode != CMVE_SIM_BF16X3);
}

// true when launch_sim takes the G64 ring kernel (64 x 64 tiles: problems of fewer than 128 tiles of 128^2)
static bool sim_uses_g64(int64_t nq_pad, int64_t ng_pad) {
  return sim_geo_force() != 128 && !(nq_pad % 256 == 0 && ng_pad % 256 == 0 && (nq_pad / 256) * (ng_pad / 256) >= 512) &&
         (nq_pad / 128) * (ng_pad / 128) < 128 && nq_pad % 64 == 0 && ng_pad % 64 == 0;
}

template <int MODE, int EPI>
static int launch_sim(const SimArgs& a, int64_t nq_pad, int64_t ng_pad, hipStream_t stream) {
  const int force = sim_geo_force();
  if (force != 128 && nq_pad % 256 == 0 && ng_pad % 256 == 0 && (nq_pad / 256) * (ng_pad / 256) >= 512) {
    if constexpr (MODE != CMVE_SIM_BF16X3)  // (split-bf16 takes the phased loop only)
      if (force == 2562) return launch_geo<MODE, EPI, 2, 4, 8, false>(a, nq_pad, ng_pad, stream);  // 2-stage BK64
    return launch_geo<MODE, EPI, 2, 4, 8, true>(a, nq_pad, ng_pad, stream);
  }
  // G64 (4 waves of 16 x 64, 64 x 64 tiles) when the 128^2 grid would leave most CUs idle (a 1k x 1k
  // problem: 64 tiles of 128^2 vs 256 of 64^2); every output element sees the same MFMA sequence in every
  // geometry.  4 waves rather than 2 of 32 x 64: the rank epilogue's scoring runs on all 4 SIMDs (2.0 ->
  // 1.2 us per tile in the K14 stamps); the main loop stays at ~6.3 us (the CU's L2 -> LDS fill of 256 KiB)
  if (force != 128 && (nq_pad / 128) * (ng_pad / 128) < 128 && nq_pad % 64 == 0 && ng_pad % 64 == 0) {
#ifndef CMVE_G64_2W
    // the rank GEMM at this size (one K14 evaluation, cmve_rank_mfma of a 1k x 1k problem): its 256 tiles are one per
    // CU, each a latency chain of 16 K-tiles -- two K groups of 4 waves halve the chain (and share the K14 level-2
    // re-score): one evaluation 31.6 -> 29.2 us back to back (profiles/r06_ab_g64_kg2.txt).  Every G64 rank launch
    // takes it, so the separate-launch path and cmve_eval_ranks still see the same scores (CMVE_G64_KG = 1: off)
    if constexpr (EPI == EPI_RANK && MODE != CMVE_SIM_BF16X3 && CMVE_G64_KG == 2)
      if (a.nk0 >= 2 && a.nk0 % 2 == 0) return launch_geo<MODE, EPI, 4, 1, 1, false, 2>(a, nq_pad, ng_pad, stream);
    return launch_geo<MODE, EPI, 4, 1, 1, false>(a, nq_pad, ng_pad, stream);
#else
    return launch_geo<MODE, EPI, 2, 1, 2, false>(a, nq_pad, ng_pad, stream);
#endif
  }
  return launch_geo<MODE, EPI, 2, 2, 4, false>(a, nq_pad, ng_pad, stream);
}

static int validate_pair(const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, const char* fn) {
  CMVE_REQUIRE(q && g, "%s: NULL rows", fn);
  CMVE_REQUIRE(q->d == g->d && q->d_pad == g->d_pad, "%s: dimension mismatch (%lld vs %lld)", fn, (long long)q->d,
               (long long)g->d);
  CMVE_REQUIRE(q->n_pad % 128 == 0 && g->n_pad % 128 == 0 && q->d_pad % BK == 0, "%s: sets not packed/padded", fn);
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
  a.nk0 = (int)(q->d_pad / BK);
  a.nk = mode == CMVE_SIM_BF16X3 ? 3 * a.nk0 : a.nk0;
  return a;
}

template <int EPI>
static int dispatch(const SimArgs& a, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, hipStream_t s) {
  if (mode == CMVE_SIM_BF16) return launch_sim<CMVE_SIM_BF16, EPI>(a, q->n_pad, g->n_pad, s);
  if (mode == CMVE_SIM_F16) return launch_sim<CMVE_SIM_F16, EPI>(a, q->n_pad, g->n_pad, s);
  return launch_sim<CMVE_SIM_BF16X3, EPI>(a, q->n_pad, g->n_pad, s);
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
  return dispatch<EPI_STORE>(a, q, g, mode, h->stream);
}

// defined in rank.hip
namespace cmve {
int launch_cand_finalize(hipStream_t stream, const cmve_rows_t* g, uint64_t* cand, int64_t cand_cap,
                         int64_t* cand_count);
int launch_fixup(hipStream_t stream, const cmve_rows_t* q, const cmve_rows_t* g, int32_t dirs, const double* row_sgt,
                 const double* col_sgt, int32_t* row_cnt, int32_t* col_cnt, const uint64_t* cand, int64_t cand_cap,
                 const int64_t* cand_count);
}

// point the epilogue at the bucketed layout of `cand` (cand_layout) for the gallery view g
static void set_cand(SimArgs& a, const cmve_rows_t* g, uint64_t* cand, int64_t cand_cap, int64_t* cand_count) {
  const CandLayout l = cand_layout(g->n_pad, cand_cap);
  a.bucket_cnt = (unsigned long long*)cand;
  a.cand = (unsigned long long*)(cand + l.nb);
  a.cap_b = l.cap_b;
  a.cand_cap = cand_cap;
  a.cand_count = (unsigned long long*)cand_count;
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
  CMVE_REQUIRE(!((q->flags | g->flags) & CMVE_PACK_RAW), "%s: sets packed CMVE_PACK_RAW have no score bound", fn);
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
  set_cand(a, g, cand, cand_cap, cand_count);
  return CMVE_OK;
}

// zero the bucket counters, run the rank GEMM, then write the pair total (or an overflow size) to
// *cand_count.  A buffer too small for the bucket counters is reported as overflow untouched.
static int rank_pass(const SimArgs& a, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, uint64_t* cand,
                     int64_t cand_cap, int64_t* cand_count, hipStream_t s) {
  const CandLayout l = cand_layout(g->n_pad, cand_cap);
  if (l.cap_b == 0) return launch_cand_finalize(s, g, nullptr, cand_cap, cand_count);
  CMVE_HIP(hipMemsetAsync(cand, 0, sizeof(uint64_t) * l.nb, s));
  int st = dispatch<EPI_RANK>(a, q, g, mode, s);
  if (st) return st;
  return launch_cand_finalize(s, g, cand, cand_cap, cand_count);
}

namespace cmve {
// K13 main pass (topk.hip): the TOPK epilogue over the whole gallery with per-row thresholds
// (hi, lo) = (+inf, tau); entries land in cand[nb + b * cap_b ...], b = query row >> 8, counters
// in cand[0, nb) (zeroed by the caller)
int launch_topk_gemm(hipStream_t s, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, const float* row_hi,
                     const float* row_lo, uint64_t* cand, int64_t nb, int64_t cap_b) {
  int st = validate_pair(q, g, mode, "cmve_topk_batch");
  if (st) return st;
  CMVE_REQUIRE(q->n_pad <= (int64_t)nb * 256, "cmve_topk_batch: bucket count too small");
  CMVE_REQUIRE(g->n < (1ll << 24), "cmve_topk_batch: gallery shard must hold < 2^24 rows");
  SimArgs a = make_args(q, g, mode);
  a.row_hi = row_hi;
  a.row_lo = row_lo;
  a.bucket_cnt = (unsigned long long*)cand;
  a.cand = (unsigned long long*)(cand + nb);
  a.cap_b = cap_b;
  return dispatch<EPI_TOPK>(a, q, g, mode, s);
}
}  // namespace cmve

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
  return rank_pass(a, q, g, mode, cand, cand_cap, cand_count, h->stream);
}

extern "C" int cmve_rank_fixup(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t dirs,
                               const double* row_sgt, const double* col_sgt, int32_t* row_cnt, int32_t* col_cnt,
                               const uint64_t* cand, int64_t cand_cap, const int64_t* cand_count) {
  CMVE_REQUIRE(h && q && g, "cmve_rank_fixup: NULL argument");
  CMVE_REQUIRE(q->d == g->d, "cmve_rank_fixup: dimension mismatch");
  if (dirs & CMVE_DIR_ROW) CMVE_REQUIRE(row_sgt && row_cnt, "cmve_rank_fixup: row arrays missing");
  if (dirs & CMVE_DIR_COL) CMVE_REQUIRE(col_sgt && col_cnt, "cmve_rank_fixup: col arrays missing");
  CMVE_REQUIRE(cand && cand_count, "cmve_rank_fixup: candidate buffer missing");
  if (q->n == 0 || g->n == 0) return CMVE_OK;  // nothing to re-score (an empty gallery shard)
  CMVE_REQUIRE(q->raw && g->raw && q->inv_norm && g->inv_norm, "cmve_rank_fixup: raw rows / norms missing");
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

static size_t elem_bytes(int32_t dt) { return (dt == CMVE_F64 || dt == CMVE_I64) ? 8 : dt == CMVE_BF16 ? 2 : 4; }

// rows [r0, r0 + rows_pad) of a packed set as a packed set of its own (err_max stays the whole
// set's: a valid, slightly looser bound for the chunk)
static cmve_rows_t chunk_view(const cmve_rows_t* g, int64_t r0, int64_t rows_pad) {
  cmve_rows_t v = *g;
  v.n = std::max<int64_t>(0, std::min<int64_t>(g->n - r0, rows_pad));
  v.n_pad = rows_pad;
  const int64_t e = r0 * g->d_pad;
  if (g->hi) v.hi = g->hi + e;
  if (g->lo) v.lo = g->lo + e;
  if (g->h16) v.h16 = g->h16 + e;
  if (g->raw) v.raw = (const char*)g->raw + r0 * g->raw_ld * (int64_t)elem_bytes(g->raw_dtype);
  if (g->inv_norm) v.inv_norm = g->inv_norm + r0;
  if (g->err_hi) v.err_hi = g->err_hi + r0;
  if (g->err_hilo) v.err_hilo = g->err_hilo + r0;
  if (g->err_h16) v.err_h16 = g->err_h16 + r0;
  return v;
}

static int ensure_aux(cmve_handle_t h) {
  if (h->aux) return CMVE_OK;
  int cur = 0;
  CMVE_HIP(hipGetDevice(&cur));
  CMVE_HIP(hipSetDevice(h->device));
  hipError_t e = hipStreamCreateWithFlags(&h->aux, hipStreamNonBlocking);
  for (int i = 0; e == hipSuccess && i < CMVE_MAX_CHUNKS + 2; ++i)
    e = hipEventCreateWithFlags(&h->ev[i], hipEventDisableTiming);
  for (int i = 0; e == hipSuccess && i < 2 * CMVE_MAX_CHUNKS; ++i) e = hipEventCreate(&h->tev[i]);
  (void)hipSetDevice(cur);
  CMVE_HIP(e);
  return CMVE_OK;
}

extern "C" int cmve_rank_count_overlap(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode,
                                       int32_t dirs, const double* row_sgt, const float* row_hi, const float* row_lo,
                                       const double* col_sgt, const float* col_hi, const float* col_lo,
                                       int32_t* row_cnt, int32_t* col_cnt, uint64_t* cand, int64_t cand_cap,
                                       int64_t* cand_count, int32_t chunks) {
  CMVE_REQUIRE(h, "cmve_rank_count_overlap: NULL handle");
  CMVE_REQUIRE(chunks >= 1 && chunks <= CMVE_MAX_CHUNKS, "cmve_rank_count_overlap: chunks must be in [1, %d]",
               CMVE_MAX_CHUNKS);
  if (dirs & CMVE_DIR_ROW) CMVE_REQUIRE(row_sgt, "cmve_rank_count_overlap: row_sgt missing");
  if (dirs & CMVE_DIR_COL) CMVE_REQUIRE(col_sgt, "cmve_rank_count_overlap: col_sgt missing");
  SimArgs a;
  int st = rank_args(q, g, mode, dirs, row_hi, row_lo, col_hi, col_lo, row_cnt, col_cnt, cand, cand_cap, cand_count,
                     a, "cmve_rank_count_overlap");
  if (st) return st;
  hipStream_t s0 = h->stream;
  CMVE_HIP(hipMemsetAsync(cand_count, 0, sizeof(int64_t) * chunks, s0));
  if (dirs & CMVE_DIR_ROW) CMVE_HIP(hipMemsetAsync(row_cnt, 0, sizeof(int32_t) * q->n_pad, s0));
  if (dirs & CMVE_DIR_COL) CMVE_HIP(hipMemsetAsync(col_cnt, 0, sizeof(int32_t) * g->n_pad, s0));
  if (q->n == 0 || g->n == 0) return CMVE_OK;
  CMVE_REQUIRE(q->raw && g->raw && q->inv_norm && g->inv_norm, "cmve_rank_count_overlap: raw rows / norms missing");
  st = ensure_aux(h);
  if (st) return st;
  // chunk rows: a multiple of CMVE_ROW_ALIGN covering g->n_pad in `chunks` pieces
  const int64_t units = g->n_pad / CMVE_ROW_ALIGN;
  const int64_t per = ((units + chunks - 1) / chunks) * CMVE_ROW_ALIGN;
  const int64_t cap_c = cand_cap / chunks;
  CMVE_HIP(hipEventRecord(h->ev[0], s0));
  CMVE_HIP(hipStreamWaitEvent(h->aux, h->ev[0], 0));
  int used = 0;
  for (int c = 0; c < chunks; ++c) {
    const int64_t r0 = (int64_t)c * per;
    if (r0 >= g->n) break;
    const cmve_rows_t v = chunk_view(g, r0, std::min<int64_t>(per, g->n_pad - r0));
    SimArgs ac = a;
    ac.ghi = mode == CMVE_SIM_F16 ? v.h16 : v.hi;
    ac.glo = v.lo;
    ac.ng = (int)v.n;
    if (dirs & CMVE_DIR_COL) {
      ac.col_hi = col_hi + r0;
      ac.col_lo = col_lo + r0;
      ac.col_cnt = col_cnt + r0;
    }
    set_cand(ac, &v, cand + c * cap_c, cap_c, cand_count + c);
    CMVE_HIP(hipEventRecord(h->tev[2 * c], s0));
    st = rank_pass(ac, q, &v, mode, cand + c * cap_c, cap_c, cand_count + c, s0);
    if (st) return st;
    CMVE_HIP(hipEventRecord(h->tev[2 * c + 1], s0));
    CMVE_HIP(hipEventRecord(h->ev[1 + c], s0));
    CMVE_HIP(hipStreamWaitEvent(h->aux, h->ev[1 + c], 0));
    st = launch_fixup(h->aux, q, &v, dirs, row_sgt, (dirs & CMVE_DIR_COL) ? col_sgt + r0 : nullptr, row_cnt,
                      (dirs & CMVE_DIR_COL) ? col_cnt + r0 : nullptr, cand + c * cap_c, cap_c, cand_count + c);
    if (st) return st;
    used = c + 1;
  }
  h->last_chunks = used;
  CMVE_HIP(hipEventRecord(h->ev[CMVE_MAX_CHUNKS + 1], h->aux));
  CMVE_HIP(hipStreamWaitEvent(s0, h->ev[CMVE_MAX_CHUNKS + 1], 0));
  return CMVE_OK;
}

extern "C" int cmve_overlap_mfma_ms(cmve_handle_t h, float* ms, int32_t* launches) {
  CMVE_REQUIRE(h && ms && launches, "cmve_overlap_mfma_ms: NULL argument");
  *ms = 0.f;
  *launches = h->last_chunks;
  for (int c = 0; c < h->last_chunks; ++c) {
    float t = 0.f;
    CMVE_HIP(hipEventSynchronize(h->tev[2 * c + 1]));
    CMVE_HIP(hipEventElapsedTime(&t, h->tev[2 * c], h->tev[2 * c + 1]));
    *ms += t;
  }
  return CMVE_OK;
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
  CMVE_REQUIRE(relu >= 0 && relu <= 3, "cmve_linear: unknown activation %d", relu);
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
  if (!resid && !bn_scale && relu <= 1) return dispatch<EPI_BIAS>(a, x, w, mode, h->stream);
  return dispatch<EPI_LINEAR>(a, x, w, mode, h->stream);
}

// ---- K14: the three-launch evaluation (eval.hip) ----
#include "eval_abi.h"

namespace {
struct EvalWs {
  size_t done, q_sgt, q_hi, q_lo, q_cnt, g_sgt, g_hi, g_lo, g_cnt, q_gt1, g_gt1, q_el, g_el, q_l16, g_l16, l3, cand,
      total;
};
// the lo16 planes: [n_pad, d_pad] bf16 each side, the level-2 re-score's residuals (lo16_elem); l3: the level-3
// list (a count word, then EVAL_L3_CAP entries)
constexpr int EVAL_L3_CAP = 4096;
EvalWs eval_ws_layout(int64_t nq_pad, int64_t ng_pad, int64_t d_pad, int64_t cand_cap) {
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  EvalWs w;
  size_t o = 0;
  w.done = o;
  o = up(o + 2 * sizeof(unsigned) * cmve::EVAL_ARRIVAL_WORDS);
  w.q_sgt = o;
  o = up(o + 8 * (size_t)nq_pad);
  w.q_hi = o;
  o = up(o + 4 * (size_t)nq_pad);
  w.q_lo = o;
  o = up(o + 4 * (size_t)nq_pad);
  w.q_cnt = o;
  o = up(o + 4 * (size_t)nq_pad);
  w.g_sgt = o;
  o = up(o + 8 * (size_t)ng_pad);
  w.g_hi = o;
  o = up(o + 4 * (size_t)ng_pad);
  w.g_lo = o;
  o = up(o + 4 * (size_t)ng_pad);
  w.g_cnt = o;
  o = up(o + 4 * (size_t)ng_pad);
  w.q_gt1 = o;
  o = up(o + 4 * (size_t)nq_pad);
  w.g_gt1 = o;
  o = up(o + 4 * (size_t)ng_pad);
  w.q_el = o;
  o = up(o + 4 * (size_t)nq_pad);
  w.g_el = o;
  o = up(o + 4 * (size_t)ng_pad);
  w.q_l16 = o;
  o = up(o + 2 * (size_t)nq_pad * (size_t)d_pad);
  w.g_l16 = o;
  o = up(o + 2 * (size_t)ng_pad * (size_t)d_pad);
  w.l3 = o;
  o = up(o + 8 + 8 * (size_t)EVAL_L3_CAP);
  w.cand = o;
  o = up(o + 8 * (size_t)cand_cap);
  w.total = o;
  return w;
}
}  // namespace

static unsigned long long* g_eval_stamps = nullptr;
// kernel studies only (not in cmve.h): copy the last CMVE_EVAL_DBG & 128 stamps to the host
extern "C" int cmve_eval_debug_stamps(void* host, int64_t bytes) {
  CMVE_REQUIRE(g_eval_stamps && host, "cmve_eval_debug_stamps: no stamps (CMVE_EVAL_DBG & 128)");
  CMVE_HIP(hipDeviceSynchronize());
  CMVE_HIP(hipMemcpy(host, g_eval_stamps, std::min<int64_t>(bytes, sizeof(unsigned long long) * 4 * 1024 * 8),
                     hipMemcpyDeviceToHost));
  return CMVE_OK;
}

extern "C" int cmve_eval_workspace(const cmve_rows_t* q, const cmve_rows_t* g, int64_t cand_cap, int64_t* bytes) {
  CMVE_REQUIRE(q && g && bytes, "cmve_eval_workspace: NULL argument");
  CMVE_REQUIRE(cand_cap > 0, "cmve_eval_workspace: cand_cap must be > 0");
  *bytes = (int64_t)eval_ws_layout(q->n_pad, g->n_pad, q->d_pad, cand_cap).total;
  return CMVE_OK;
}

static cmve::EvalSide eval_side(cmve_rows_t* r, const int64_t* off, const int32_t* idx, char* ws, size_t o_sgt,
                                size_t o_hi, size_t o_lo, size_t o_cnt, size_t o_gt1, int64_t* ranks) {
  cmve::EvalSide s{};
  s.raw = r->raw;
  s.ld = r->raw_ld;
  s.n = r->n;
  s.n_pad = r->n_pad;
  s.vec = r->raw_dtype == CMVE_F32 ? rows_vec4((const float*)r->raw, r->d, r->raw_ld)
                                    : rows_vec4((const double*)r->raw, r->d, r->raw_ld);
  s.flags = r->flags;
  s.eps = r->eps;
  s.hi = r->hi;
  s.lo = r->lo;
  s.h16 = r->h16;
  s.inv = r->inv_norm;
  s.err_hi = r->err_hi;
  s.err_hilo = r->err_hilo;
  s.err_h16 = r->err_h16;
  s.err_max = r->err_max;
  s.off = off;
  s.idx = idx;
  s.sgt = (double*)(ws + o_sgt);
  s.thr_hi = (float*)(ws + o_hi);
  s.thr_lo = (float*)(ws + o_lo);
  s.cnt = (int32_t*)(ws + o_cnt);
  s.gt1 = off ? (int32_t*)(ws + o_gt1) : nullptr;
  s.ranks = ranks;
  return s;
}

// K14 at G256 sizes: the persistent rank kernel reads explicit thresholds, so they are written here by
// the rule the 2-stage / ring kernels apply in-kernel (sim_kernel's thr_of: the other set's err_max
// folded from the prep's shards, then gt_thr_kernel's directed rounding); one thread per row of either set
struct EvalThrSide {
  const double* sgt;
  const float* err;
  const unsigned* emax_other;
  float* hi;
  float* lo;
  int64_t n_pad;
};
__global__ __launch_bounds__(256) void eval_thr_kernel(EvalThrSide s0, EvalThrSide s1, int64_t d_pad, int mode) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool first = r < s0.n_pad;
  const EvalThrSide& s = first ? s0 : s1;
  if (!first) r -= s0.n_pad;
  if (!s.hi || r >= s.n_pad) return;
  unsigned m = 0u;
  for (int k = 0; k < EVAL_EMAX_SHARDS; ++k) m = max(m, s.emax_other[k]);
  const double E = score_error_bound((double)s.err[r], (double)__uint_as_float(m), d_pad, mode);
  const double sgt = s.sgt[r];  // NaN (no GT, padding) or +inf (every GT NaN): never counted
  s.hi[r] = sgt < INFINITY ? f32_round_up(sgt + E) : INFINITY;
  s.lo[r] = sgt < INFINITY ? f32_round_down(sgt - E) : INFINITY;
}

// Everything of one K14 evaluation but its launches: argument checks, the workspace layout and the argument
// blocks of the prep / rank GEMM / fix-up / finish launches (cmve_eval_ranks launches them at once;
// cmve_eval_batch_create stores them in a device table)
struct EvalPlan {
  cmve::EvalSide sq, sg;
  cmve::EvalCommon c;
  SimArgs a;
  int qf, gf;
  bool paired, inline_fix;
  bool fix_launch = false;  // (inline_fix sizes) the GEMM lists its undecided pairs for a fix-up launch (level 2 + fp64)
};

static int eval_prepare(cmve_rows_t* q, cmve_rows_t* g, int32_t mode_flags, const int64_t* row_off,
                        const int32_t* row_idx, const int64_t* col_off, const int32_t* col_idx, void* ws,
                        int64_t ws_bytes, int64_t cand_cap, int64_t* out, const char* fn, EvalPlan& P,
                        bool batch = false) {
  const int32_t mode = mode_flags & 0xff;
  const bool paired_req = (mode_flags & CMVE_EVAL_PAIRED) != 0;
  CMVE_REQUIRE((mode_flags & ~(0xff | CMVE_EVAL_PAIRED)) == 0, "%s: unknown flags 0x%x", fn, mode_flags);
  int st = validate_pair(q, g, mode, fn);
  if (st) return st;
  CMVE_REQUIRE(q->n > 0 && g->n > 0, "%s: both sets need rows", fn);
  CMVE_REQUIRE(q->raw && g->raw && q->inv_norm && g->inv_norm && q->err_hi && q->err_hilo && g->err_hi &&
                   g->err_hilo && q->err_max && g->err_max,
               "%s: packed-set arrays missing", fn);
  CMVE_REQUIRE(!((q->flags | g->flags) & CMVE_PACK_RAW), "%s: sets packed CMVE_PACK_RAW have no score bound", fn);
  CMVE_REQUIRE((q->raw_dtype == CMVE_F32 || q->raw_dtype == CMVE_F64) &&
                   (g->raw_dtype == CMVE_F32 || g->raw_dtype == CMVE_F64),
               "%s: raw rows must be F32 or F64", fn);
  CMVE_REQUIRE(q->raw_ld >= q->d && g->raw_ld >= g->d, "%s: raw_ld < d", fn);
  CMVE_REQUIRE((q->h16 == nullptr) == (q->err_h16 == nullptr) && (g->h16 == nullptr) == (g->err_h16 == nullptr),
               "%s: h16 and err_h16 go together", fn);
  CMVE_REQUIRE((row_off != nullptr) == (row_idx != nullptr) && (col_off != nullptr) == (col_idx != nullptr),
               "%s: GT offsets and indices go together", fn);
  CMVE_REQUIRE(row_off || col_off, "%s: no direction requested", fn);
  CMVE_REQUIRE(ws && out, "%s: NULL workspace / output", fn);
  const EvalWs w = eval_ws_layout(q->n_pad, g->n_pad, q->d_pad, cand_cap);
  CMVE_REQUIRE(cand_cap > 0 && ws_bytes >= (int64_t)w.total, "%s: workspace has %lld bytes, needs %lld", fn,
               (long long)ws_bytes, (long long)w.total);
  CandLayout l = cand_layout(g->n_pad, cand_cap);
  // one bucket per 64 x 64 output tile when the grid is small: each wave reserves its undecided-pair
  // slots on its own tile's counter (by 256 gallery rows a 1k x 1k evaluation has 4 counters, ~125
  // serialised returning atomics each); the fix-up walks them flat
  const int64_t nb_tiles = (q->n_pad >> 6) * (g->n_pad >> 6);
  const bool tile_buckets = nb_tiles <= FIXUP_MAX_BUCKETS_PER_XCD && cand_cap >= 8 * nb_tiles;
  if (tile_buckets) {
    l.nb = nb_tiles;
    l.cap_b = (cand_cap - nb_tiles) / nb_tiles;
  }
  CMVE_REQUIRE(l.cap_b > 0, "%s: cand_cap %lld cannot hold the %lld bucket counters", fn, (long long)cand_cap,
               (long long)l.nb);
  CMVE_REQUIRE((l.nb + 7) / 8 <= FIXUP_MAX_BUCKETS_PER_XCD, "%s: gallery set too large (%lld buckets)", fn,
               (long long)l.nb);
  char* base = (char*)ws;
  P.sq = eval_side(q, row_off, row_idx, base, w.q_sgt, w.q_hi, w.q_lo, w.q_cnt, w.q_gt1, out + CMVE_EVAL_OUT_HEAD);
  P.sg = eval_side(g, col_off, col_idx, base, w.g_sgt, w.g_hi, w.g_lo, w.g_cnt, w.g_gt1,
                   out + CMVE_EVAL_OUT_HEAD + q->n);
  cmve::EvalCommon& c = P.c;
  c = cmve::EvalCommon{};
  c.d = q->d;
  c.d_pad = q->d_pad;
  c.mode = mode;
  c.emax = (unsigned*)(base + w.done);
  uint64_t* cand = (uint64_t*)(base + w.cand);
  c.bucket = (unsigned long long*)cand;
  c.nb = l.nb;
  c.cap_b = l.cap_b;
  c.cand = cand;
  c.stats = out;
  constexpr int dbg = CMVE_EVAL_DBG;  // kernel studies only (a study build)
  c.dbg = dbg;
  static unsigned long long* stamp_buf = nullptr;
  if ((dbg & 128) && !stamp_buf) {
    CMVE_HIP(hipMalloc(&stamp_buf, sizeof(unsigned long long) * 4 * 1024 * 8));
    CMVE_HIP(hipMemset(stamp_buf, 0, sizeof(unsigned long long) * 4 * 1024 * 8));
  }
  c.stamps = (dbg & 128) ? stamp_buf : nullptr;
  g_eval_stamps = c.stamps;
  P.qf = q->raw_dtype == CMVE_F64;
  P.gf = g->raw_dtype == CMVE_F64;
  if (paired_req)
    CMVE_REQUIRE(row_off && col_off && q->n == g->n && q->n_pad == g->n_pad,
                 "%s: CMVE_EVAL_PAIRED needs both directions and equal set sizes", fn);
  // the paired prep reads rows through the register path only (16-B pieces, d_pad <= 1024)
  P.paired = paired_req && P.sq.vec && P.sg.vec && q->d_pad <= 1024;
  SimArgs& a = P.a;
  a = make_args(q, g, mode);
  // thresholds derived in the GEMM from the prep's GT scores and per-row bounds (row_hi / col_hi only
  // mark the directions that are on)
  a.thr_gt = !sim_uses_phased(mode, q->n_pad, g->n_pad);
  a.q_err = mode_err(q, mode);
  a.g_err = mode_err(g, mode);
  a.q_emax = c.emax + (0 * 3 + mode_slot(mode)) * cmve::EMAX_SHARDS;
  a.g_emax = c.emax + (1 * 3 + mode_slot(mode)) * cmve::EMAX_SHARDS;
  if (row_off) {
    a.row_hi = P.sq.thr_hi;
    a.row_lo = P.sq.thr_lo;
    a.row_sgt = P.sq.sgt;
    a.row_cnt = P.sq.cnt;
  }
  if (col_off) {
    a.col_hi = P.sg.thr_hi;
    a.col_lo = P.sg.thr_lo;
    a.col_sgt = P.sg.sgt;
    a.col_cnt = P.sg.cnt;
  }
  set_cand(a, g, cand, cand_cap, out + 10);  // (the epilogue never writes cand_count)
  a.bucket_cnt = (unsigned long long*)cand;  // the evaluation's layout (l: per-tile buckets when small)
  a.cand = (unsigned long long*)(cand + l.nb);
  a.cap_b = l.cap_b;
  a.tile_buckets = tile_buckets;
  a.nbn64 = (int)(g->n_pad >> 6);
  if (a.thr_gt) {  // (the 2-stage / ring kernels; the persistent G256 kernel keeps every undecided pair)
    a.row_gt1 = P.sq.gt1;
    a.col_gt1 = P.sg.gt1;
  }
  // G64 (1k-A scale): the rank GEMM re-scores its own undecided pairs (no list, no fix-up launch)
  P.inline_fix = a.thr_gt && sim_uses_g64(q->n_pad, g->n_pad);
  // level-2 re-score from the fp16 + bf16 residual planes: the F16 mode whose prep runs the register path (the
  // only one that writes lo16: 16-B row pieces, d_pad <= 1024, both sides).  Two forms: (a) inline (the default)
  // -- level 2 inside the rank GEMM, level 3 deferred to the finish through the workspace's list; (b) the fix-up
  // launch (CMVE_EVAL_INLINE_L2=0, kernel studies) -- the rank GEMM only lists its undecided pairs and eval_fix
  // re-scores them, two pairs per wave.  Measured (round 4, tools/ab_env.sh, batches of 8): (b) takes the round
  // trips out of the GEMM (38 -> 27 us) but its own launch costs 27 us -- its gathers miss the L2 the GEMM's
  // tiles had just filled -- and a single evaluation pays a launch boundary (b2b 35.0 vs 35.9 us).
  // Study builds: CMVE_EVAL_INLINE_L2=0 (form b), CMVE_EVAL_NO_L2=1 (every band pair in fp64 inside the GEMM)
  constexpr bool no_l2 = CMVE_EVAL_NO_L2 != 0;
  constexpr bool inline_l2 = CMVE_EVAL_INLINE_L2 != 0;
  // level 3 of ONE evaluation (cmve_eval_ranks, its graphs): re-scored inside the rank GEMM (its ~4 pairs cost the
  // GEMM ~0.7 us and spare the finish its fp64 round trip, 5.2 -> 4.4 us: 32.5 -> 31.4 us back to back); batches list
  // them for the finish (in a chained run it rides in the next prep launch).  Both count them (out[12]).
  // Study builds: CMVE_EVAL_L3_LIST=1, the single evaluation lists them too
  const bool l3_inline = !batch && CMVE_EVAL_L3_LIST == 0;
  const bool l2 = P.inline_fix && mode == CMVE_SIM_F16 && P.sq.vec && P.sg.vec && q->d_pad <= 1024 && !no_l2;
  P.fix_launch = l2 && !inline_l2;
  if (l2) {
    P.sq.lo16 = (uint16_t*)(base + w.q_l16);
    P.sg.lo16 = (uint16_t*)(base + w.g_l16);
    P.sq.err_lo16 = (float*)(base + w.q_el);
    P.sg.err_lo16 = (float*)(base + w.g_el);
    a.q_lo16 = P.sq.lo16;
    a.g_lo16 = P.sg.lo16;
    a.q_el = P.sq.err_lo16;
    a.g_el = P.sg.err_lo16;
    if (!P.fix_launch) {
      c.l3_count = (unsigned*)(base + w.l3);
      c.l3 = (uint64_t*)(base + w.l3 + 8);
      c.l3_cap = l3_inline ? 0 : EVAL_L3_CAP;  // (0: the finish re-scores nothing; its count still reaches out[12])
      a.l3_count = c.l3_count;
      a.l3 = l3_inline ? nullptr : (unsigned long long*)c.l3;
      a.l3_cap = c.l3_cap;
    }
  }
  if (P.inline_fix) {
    // fix_inline 1: the GEMM re-scores its undecided pairs; with the fix-up launch (2) it lists them and re-scores
    // only the pairs of a wave whose bucket is full (SimArgs::ovf_inline): never an overflow either way
    a.fix_inline = P.fix_launch ? 0 : 1;
    a.ovf_inline = P.fix_launch ? 1 : 0;
    a.q_f64 = P.qf;
    a.g_f64 = P.gf;
    a.q_raw = q->raw;
    a.g_raw = g->raw;
    a.q_ld = q->raw_ld;
    a.g_ld = g->raw_ld;
    a.d = q->d;
    a.q_inv = q->inv_norm;
    a.g_inv = g->inv_norm;
    c.fix_inline = P.fix_launch ? 2 : 1;
  }
  a.dbg_stamps = c.stamps ? c.stamps + 3 * 1024 * 8 : nullptr;
  return CMVE_OK;
}

extern "C" int cmve_eval_ranks(cmve_handle_t h, cmve_rows_t* q, cmve_rows_t* g, int32_t mode_flags,
                               const int64_t* row_off, const int32_t* row_idx, const int64_t* col_off,
                               const int32_t* col_idx, void* ws, int64_t ws_bytes, int64_t cand_cap, int64_t* out,
                               int32_t timing_slot) {
  CMVE_REQUIRE(h, "cmve_eval_ranks: NULL handle");
  CMVE_REQUIRE(timing_slot >= -1 && timing_slot < CMVE_EVAL_TIMING_SLOTS, "cmve_eval_ranks: bad timing slot");
  EvalPlan P;
  int st = eval_prepare(q, g, mode_flags, row_off, row_idx, col_off, col_idx, ws, ws_bytes, cand_cap, out,
                        "cmve_eval_ranks", P);
  if (st) return st;
  const int32_t mode = mode_flags & 0xff;
  hipEvent_t* ev = nullptr;
  hipEvent_t* kev = nullptr;
  if (timing_slot >= 0) {
    ev = h->eval_ev[timing_slot];
    for (int k = 0; k < 4; ++k)
      if (!ev[k]) CMVE_HIP(hipEventCreate(&ev[k]));
    kev = h->eval_kev[timing_slot];
    for (int k = 0; k < 8; ++k)
      if (!kev[k]) CMVE_HIP(hipEventCreate(&kev[k]));
  }
  auto arm = [&](int k) {  // the next launch's own start / stop (cmve::launch)
    if (kev) cmve::g_launch_ev = cmve::LaunchEv{kev[2 * k], kev[2 * k + 1]};
  };
  hipStream_t s = h->stream;
  if (ev) CMVE_HIP(hipEventRecord(ev[0], s));
  arm(0);
  st = cmve::launch_eval(P.sq, P.sg, P.c, P.qf, P.gf, P.paired ? 3 : 0, s);
  if (st) return st;
  if (ev) CMVE_HIP(hipEventRecord(ev[1], s));
  const SimArgs& a = P.a;
  if (!a.thr_gt) {
    EvalThrSide t0{a.row_sgt, a.q_err, a.g_emax, row_off ? P.sq.thr_hi : nullptr, P.sq.thr_lo, q->n_pad};
    EvalThrSide t1{a.col_sgt, a.g_err, a.q_emax, col_off ? P.sg.thr_hi : nullptr, P.sg.thr_lo, g->n_pad};
    const int64_t nthr = q->n_pad + g->n_pad;
    hipLaunchKernelGGL(eval_thr_kernel, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, s, t0, t1, q->d_pad,
                       (int)mode);
    st = check_launch("eval_thr_kernel");
    if (st) return st;
  }
  arm(1);
  st = dispatch<EPI_RANK>(a, q, g, mode, s);
  if (st) return st;
  if (ev) CMVE_HIP(hipEventRecord(ev[2], s));
  if (timing_slot >= 0) {
    h->eval_no_fix[timing_slot] = P.inline_fix && !P.fix_launch;
    h->eval_chained[timing_slot] = false;
  }
  if (!P.inline_fix || P.fix_launch) {
    arm(2);
    st = cmve::launch_eval(P.sq, P.sg, P.c, P.qf, P.gf, 1, s);
    if (st) return st;
  }
  arm(3);
  st = cmve::launch_eval(P.sq, P.sg, P.c, P.qf, P.gf, 2, s);
  if (st) return st;
  if (ev) CMVE_HIP(hipEventRecord(ev[3], s));
  return CMVE_OK;
}

// ---- K14 batches: same-shaped evaluations (MSR-VTT-1kA-sized, the G64 inline fix-up geometry) in ONE set of
// three launches, each with a grid of (blocks of one evaluation) x (evaluations): a 1k x 1k evaluation's
// launches leave most of the chip idle, a batch fills it (every launch's argument blocks in a device table).
struct cmve_eval_batch {
  int count = 0;
  int qf = 0, gf = 0, mode = 0;
  bool paired = false;
  int64_t nq_pad = 0, ng_pad = 0;
  int bm = 64, bn = 64;           // the rank tile (batch_geo_bm / _bn)
  cmve::EvalSide sq0, sg0;        // the shapes (the launch grids)
  cmve::EvalCommon c0;            // (the first evaluation's: which prep kernel applies)
  bool fix_launch = false;        // the rank GEMM lists its undecided pairs for a fix-up launch
  cmve::EvalItem* d_items = nullptr;
  SimArgs* d_args = nullptr;
  std::vector<void*> ws;          // the evaluations' workspaces and outputs: a chained run refuses a previous batch
  std::vector<void*> outs;        // sharing either (its finish runs in the same launch as this batch's prep)
  bool chainable = false;         // the specialised paired prep: the chained run fuses it with the previous finish
  bool pending = false;           // its last run was chained and its finish has not been enqueued yet ...
  hipStream_t pending_stream = nullptr;  // ... on this stream (the next chained run there, or cmve_eval_batch_finish)
};

// the batch's rank geometry: 128 x 128 tiles on 4 waves of 64 x 64 (a 2-stage ring of 32 KiB stages, two blocks of
// ~73 KiB per CU, up to 256 VGPRs).  A batch's launch runs beside the other streams' launches (three batches in flight):
// a rank-GEMM block of 4 waves at 152 VGPRs leaves each SIMD room for two waves of another stream's prep, which the
// 8-wave form (round 4: 8 waves of 32 x 64 at 114 VGPRs, four waves per SIMD, 456 of 512 VGPRs) left none -- alone
// it is slower (42 vs 36 us per batch of 8), beside the preps the headline gains 4-5% (1.18 vs 1.13e11 pairs/s,
// round 5).  Split-bf16 (whose ring holds both planes) takes 128 x 64; kernel studies: CMVE_BATCH_GEO = 1288 (the
// 8-wave 128 x 128), 256128 (256 x 128, one block per CU), 64 / 12864 (64 x 64 / 128 x 64).
static constexpr int batch_geo_force() { return CMVE_BATCH_GEO; }
static bool batch_geo_big(int64_t nq_pad, int64_t ng_pad, int mode) {
  return batch_geo_force() == 256128 && nq_pad % 256 == 0 && ng_pad % 128 == 0 && mode != CMVE_SIM_BF16X3;
}
static int batch_geo_bm(int64_t nq_pad, int64_t ng_pad, int mode) {
  if (batch_geo_big(nq_pad, ng_pad, mode)) return 256;
  return (batch_geo_force() != 64 && nq_pad % 128 == 0) ? 128 : 64;
}
static int batch_geo_bn(int64_t nq_pad, int64_t ng_pad, int mode) {
  const int f = batch_geo_force();
  if (batch_geo_big(nq_pad, ng_pad, mode)) return 128;
  return (f != 64 && f != 12864 && nq_pad % 128 == 0 && ng_pad % 128 == 0 && mode != CMVE_SIM_BF16X3) ? 128 : 64;
}

template <int MODE, int WN, int TM, int WM = 4>
static int launch_rank_batch(const SimArgs* tab, int count, int64_t nq_pad, int64_t ng_pad,
                             hipStream_t stream) {
  using G = Geo<WM, WN, TM>;
  const size_t lds = (size_t)ring_stages<MODE, G::BM, G::BN, false, G::NW>() *
                     stage_bytes<MODE, G::BM, G::BN, false, kernel_kb<MODE, G::BM, G::BN, false, G::NW, true>()>();
  static const hipError_t attr_err = hipFuncSetAttribute(
      (const void*)sim_kernel<MODE, EPI_RANK, WM, WN, TM, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)lds);
  CMVE_HIP(attr_err);
  const unsigned nblocks = (unsigned)((nq_pad / G::BM) * (ng_pad / G::BN));
  cmve::launch(sim_kernel<MODE, EPI_RANK, WM, WN, TM, false, true>, dim3(nblocks, (unsigned)count), dim3(G::NT),
               (uint32_t)lds, stream, SimArgs{}, tab);
  return check_launch("sim_kernel (batch)");
}
template <int MODE>
static int launch_rank_batch(const SimArgs* tab, int count, int64_t nq_pad, int64_t ng_pad,
                             int bm, int bn, hipStream_t stream) {
  if constexpr (MODE != CMVE_SIM_BF16X3) {
    if (bm == 256 && bn == 128) return launch_rank_batch<MODE, 2, 4>(tab, count, nq_pad, ng_pad, stream);
    if (bm == 128 && bn == 128 && batch_geo_force() == 1288)  // (8 waves of 32 x 64: round 4's geometry)
      return launch_rank_batch<MODE, 2, 2>(tab, count, nq_pad, ng_pad, stream);
    if (bm == 128 && bn == 128) return launch_rank_batch<MODE, 2, 4, 2>(tab, count, nq_pad, ng_pad, stream);
  }
  return bm == 128 ? launch_rank_batch<MODE, 1, 2>(tab, count, nq_pad, ng_pad, stream)
                   : launch_rank_batch<MODE, 1, 1>(tab, count, nq_pad, ng_pad, stream);
}

extern "C" int cmve_eval_batch_create(int32_t count, cmve_rows_t* const* q, cmve_rows_t* const* g,
                                      int32_t mode_flags, const int64_t* row_off, const int32_t* row_idx,
                                      const int64_t* col_off, const int32_t* col_idx, void* const* ws,
                                      int64_t ws_bytes, int64_t cand_cap, int64_t* const* out,
                                      cmve_eval_batch_t* batch) {
  CMVE_REQUIRE(batch && q && g && ws && out && count >= 1 && count <= 65535,
               "cmve_eval_batch_create: NULL argument / count out of [1, 65535]");
  *batch = nullptr;
  std::vector<cmve::EvalItem> items((size_t)count);
  std::vector<SimArgs> args((size_t)count);
  EvalPlan P0;
  for (int i = 0; i < count; ++i) {
    EvalPlan P;
    const int st = eval_prepare(q[i], g[i], mode_flags, row_off, row_idx, col_off, col_idx, ws[i], ws_bytes,
                                cand_cap, out[i], "cmve_eval_batch_create", P, true);
    if (st) return st;
    CMVE_REQUIRE(P.inline_fix, "cmve_eval_batch_create: batches take the G64 geometry (fewer than 128 tiles of "
                               "128^2, e.g. 1,000 x 1,000) with the inline fix-up");
    if (P.c.stamps) {  // kernel studies (CMVE_EVAL_DBG & 128): the first evaluation's prep / finish blocks, and
                       // every evaluation's rank tiles while the stamp buffer's 1,024 tile slots last
      const int64_t per = (q[i]->n_pad / batch_geo_bm(q[i]->n_pad, g[i]->n_pad, mode_flags & 0xff)) *
                          (g[i]->n_pad / batch_geo_bn(q[i]->n_pad, g[i]->n_pad, mode_flags & 0xff));
      P.a.dbg_stamps = (i + 1) * per <= 1024 ? P.c.stamps + 3 * 1024 * 8 + (size_t)i * per * 8 : nullptr;
      if (i > 0) P.c.stamps = nullptr;
    }
    if (i == 0) {
      P0 = P;
    } else {
      CMVE_REQUIRE(q[i]->n == q[0]->n && g[i]->n == g[0]->n && q[i]->n_pad == q[0]->n_pad &&
                       g[i]->n_pad == g[0]->n_pad && q[i]->d == q[0]->d && q[i]->d_pad == q[0]->d_pad &&
                       P.qf == P0.qf && P.gf == P0.gf && P.paired == P0.paired,
                   "cmve_eval_batch_create: evaluation %d differs in shape / dtype / pairing from the first", i);
      // the batch's launches pick their kernels (the specialised paired prep, the level-2 re-score, a fix-up launch)
      // from the first evaluation's plan: every evaluation must plan the same way -- e.g. a row-strided input whose
      // rows are not 16-B aligned takes no register prep and no residual plane, which the specialised prep would
      // still read and write through
      CMVE_REQUIRE(P.sq.vec == P0.sq.vec && P.sg.vec == P0.sg.vec && (P.sq.lo16 != nullptr) == (P0.sq.lo16 != nullptr) &&
                       (P.sg.lo16 != nullptr) == (P0.sg.lo16 != nullptr) && P.fix_launch == P0.fix_launch &&
                       (P.c.l3_count != nullptr) == (P0.c.l3_count != nullptr),
                   "cmve_eval_batch_create: evaluation %d's inputs take another path than the first's (row alignment "
                   "or stride: every evaluation of a batch needs 16-B aligned rows if the first has them)", i);
      for (int j = 0; j < i; ++j)
        CMVE_REQUIRE(ws[j] != ws[i] && out[j] != out[i],
                     "cmve_eval_batch_create: evaluations %d and %d share a workspace or an output", j, i);
    }
    items[(size_t)i] = cmve::EvalItem{P.sq, P.sg, P.c};
    // (launch_geo fills these for a single launch)
    geo_fill(P.a, q[i]->n_pad, g[i]->n_pad, batch_geo_bm(q[i]->n_pad, g[i]->n_pad, mode_flags & 0xff),
             batch_geo_bn(q[i]->n_pad, g[i]->n_pad, mode_flags & 0xff));
    args[(size_t)i] = P.a;
  }
  auto* b = new cmve_eval_batch;
  b->count = count;
  b->qf = P0.qf;
  b->gf = P0.gf;
  b->mode = mode_flags & 0xff;
  b->paired = P0.paired;
  b->nq_pad = q[0]->n_pad;
  b->ng_pad = g[0]->n_pad;
  b->bm = batch_geo_bm(b->nq_pad, b->ng_pad, b->mode);
  b->bn = batch_geo_bn(b->nq_pad, b->ng_pad, b->mode);
  b->sq0 = P0.sq;
  b->sg0 = P0.sg;
  b->c0 = P0.c;
  b->fix_launch = P0.fix_launch;
  b->ws.assign(ws, ws + count);
  b->outs.assign(out, out + count);
  // the fused chained launch runs the specialised PAIRED prep: a batch whose lists are no one-to-one pairing (run()
  // takes the general prep, phase 0) chains through the separate finish launch instead
  b->chainable = P0.paired && cmve::eval_batch_chainable(P0.sq, P0.sg, P0.c);
  hipError_t e = hipMalloc(&b->d_items, sizeof(cmve::EvalItem) * (size_t)count);
  if (e == hipSuccess) e = hipMalloc(&b->d_args, sizeof(SimArgs) * (size_t)count);
  if (e == hipSuccess)
    e = hipMemcpy(b->d_items, items.data(), sizeof(cmve::EvalItem) * (size_t)count, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(b->d_args, args.data(), sizeof(SimArgs) * (size_t)count, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(b->d_items);
    (void)hipFree(b->d_args);
    delete b;
    CMVE_HIP(e);
  }
  *batch = b;
  return CMVE_OK;
}

// timing_slot >= 0: the three launches' own start / stop into that slot of h's ring (cmve_eval_kernel_timing:
// prep, rank GEMM, 0, finish -- durations of the whole batch's launches) and the event spans (cmve_eval_timing).
// A chained run's prep slot includes the previous batch's finish (fused into the prep launch, or its own launch)
static int eval_batch_run(cmve_handle_t h, cmve_eval_batch_t b, int32_t timing_slot, bool chained = false,
                          cmve_eval_batch_t prev = nullptr) {
  hipEvent_t* ev = nullptr;
  hipEvent_t* kev = nullptr;
  if (timing_slot >= 0) {
    ev = h->eval_ev[timing_slot];
    for (int k = 0; k < 4; ++k)
      if (!ev[k]) CMVE_HIP(hipEventCreate(&ev[k]));
    kev = h->eval_kev[timing_slot];
    for (int k = 0; k < 8; ++k)
      if (!kev[k]) CMVE_HIP(hipEventCreate(&kev[k]));
    // (the CMVE_EVAL_FIX_CHAINED study's batch has no fix-up launch of its own either)
    h->eval_no_fix[timing_slot] = !b->fix_launch || (chained && b->chainable && CMVE_EVAL_FIX_CHAINED &&
                                                     b->c0.nb <= cmve::EVAL_FIXC_MAXB);
    h->eval_chained[timing_slot] = chained;
  }
  auto arm = [&](int k) {
    if (kev) cmve::g_launch_ev = cmve::LaunchEv{kev[2 * k], kev[2 * k + 1]};
  };
  hipStream_t s = h->stream;
  int st = CMVE_OK;
  const bool fused = chained && b->chainable;  // the prep and the previous batch's finish in one launch
  // CMVE_EVAL_FIX_CHAINED study (with the fix-up launch form, CMVE_EVAL_INLINE_L2=0): the previous batch's fix-up
  // rides in this prep launch instead of following its rank GEMM; its finish then follows as a launch of its own
  const bool fchain = fused && CMVE_EVAL_FIX_CHAINED && b->fix_launch && b->c0.nb <= cmve::EVAL_FIXC_MAXB;
  if (ev) CMVE_HIP(hipEventRecord(ev[0], s));
  if (chained && prev && !fused) {  // (not the specialised prep: the previous batch's finish as a launch of its own,
    // inside the prep's timing span; its own kernel events are not taken -- slot 0's kernel pair times the prep)
    st = cmve::launch_eval_batch(prev->sq0, prev->sg0, prev->c0, prev->d_items, prev->count, prev->qf, prev->gf, 2, s);
    if (st) return st;
  }
  arm(0);
  if (fchain) {
    st = cmve::launch_eval_batch_chained(b->sq0, b->sg0, b->c0, b->d_items, nullptr, b->count, b->qf, b->gf, s,
                                         prev ? prev->d_items : nullptr);
    if (!st && prev)
      st = cmve::launch_eval_batch(prev->sq0, prev->sg0, prev->c0, prev->d_items, prev->count, prev->qf, prev->gf, 2, s);
  } else if (fused)
    st = cmve::launch_eval_batch_chained(b->sq0, b->sg0, b->c0, b->d_items, prev ? prev->d_items : nullptr, b->count,
                                         b->qf, b->gf, s);
  else
    st = cmve::launch_eval_batch(b->sq0, b->sg0, b->c0, b->d_items, b->count, b->qf, b->gf, b->paired ? 3 : 0, s);
  if (st) return st;
  if (ev) CMVE_HIP(hipEventRecord(ev[1], s));
  arm(1);
  switch (b->mode) {
    case CMVE_SIM_F16: st = launch_rank_batch<CMVE_SIM_F16>(b->d_args, b->count, b->nq_pad, b->ng_pad, b->bm, b->bn, s); break;
    case CMVE_SIM_BF16: st = launch_rank_batch<CMVE_SIM_BF16>(b->d_args, b->count, b->nq_pad, b->ng_pad, b->bm, b->bn, s); break;
    default: st = launch_rank_batch<CMVE_SIM_BF16X3>(b->d_args, b->count, b->nq_pad, b->ng_pad, b->bm, b->bn, s); break;
  }
  if (st) return st;
  if (ev) CMVE_HIP(hipEventRecord(ev[2], s));
  if (b->fix_launch && !fchain) {
    arm(2);
    st = cmve::launch_eval_batch(b->sq0, b->sg0, b->c0, b->d_items, b->count, b->qf, b->gf, 1, s);
    if (st) return st;
  }
  if (!chained) {
    arm(3);
    st = cmve::launch_eval_batch(b->sq0, b->sg0, b->c0, b->d_items, b->count, b->qf, b->gf, 2, s);
    if (st) return st;
  }
  if (ev) CMVE_HIP(hipEventRecord(ev[3], s));
  return CMVE_OK;
}

extern "C" int cmve_eval_batch_run(cmve_handle_t h, cmve_eval_batch_t b, int32_t timing_slot) {
  CMVE_REQUIRE(h && b && b->d_items && b->d_args, "cmve_eval_batch_run: NULL handle / batch");
  CMVE_REQUIRE(timing_slot >= -1 && timing_slot < CMVE_EVAL_TIMING_SLOTS, "cmve_eval_batch_run: bad timing slot");
  CMVE_REQUIRE(!b->pending, "cmve_eval_batch_run: the batch's last chained run is not finished (chain it as the previous "
                            "batch of the next chained run, or call cmve_eval_batch_finish)");
  return eval_batch_run(h, b, timing_slot);
}

extern "C" int cmve_eval_batch_run_chained(cmve_handle_t h, cmve_eval_batch_t b, cmve_eval_batch_t prev,
                                           int32_t timing_slot) {
  CMVE_REQUIRE(h && b && b->d_items && b->d_args, "cmve_eval_batch_run_chained: NULL handle / batch");
  CMVE_REQUIRE(timing_slot >= -1 && timing_slot < CMVE_EVAL_TIMING_SLOTS,
               "cmve_eval_batch_run_chained: bad timing slot");
  CMVE_REQUIRE(!b->pending, "cmve_eval_batch_run_chained: the batch's last chained run is not finished yet");
  if (prev) {
    CMVE_REQUIRE(prev->d_items && prev != b, "cmve_eval_batch_run_chained: the previous batch is destroyed or the batch itself");
    CMVE_REQUIRE(prev->pending && prev->pending_stream == h->stream,
                 "cmve_eval_batch_run_chained: the previous batch has no chained run awaiting its finish on this stream");
    CMVE_REQUIRE(prev->count == b->count && prev->nq_pad == b->nq_pad && prev->ng_pad == b->ng_pad &&
                     prev->sq0.n == b->sq0.n && prev->sg0.n == b->sg0.n && prev->qf == b->qf && prev->gf == b->gf &&
                     prev->mode == b->mode && prev->paired == b->paired && prev->chainable == b->chainable,
                 "cmve_eval_batch_run_chained: the previous batch differs in shape from the batch");
    for (void* w : b->ws)
      CMVE_REQUIRE(std::find(prev->ws.begin(), prev->ws.end(), w) == prev->ws.end(),
                   "cmve_eval_batch_run_chained: the batch shares a workspace with the previous batch, whose finish "
                   "runs in the same launch as its prep");
    // the prep zeroes out[0, 13) while the previous finish adds its R@K counts / rank sums into its own out
    const uintptr_t span = sizeof(int64_t) * (uintptr_t)(CMVE_EVAL_OUT_HEAD + b->sq0.n + b->sg0.n);
    for (void* o : b->outs)
      for (void* po : prev->outs)
        CMVE_REQUIRE((uintptr_t)o + span <= (uintptr_t)po || (uintptr_t)po + span <= (uintptr_t)o,
                     "cmve_eval_batch_run_chained: the batch shares an output with the previous batch, whose finish "
                     "runs in the same launch as its prep");
  }
  const int st = eval_batch_run(h, b, timing_slot, true, prev);
  if (st) return st;
  if (prev) prev->pending = false;
  b->pending = true;
  b->pending_stream = h->stream;
  return CMVE_OK;
}

extern "C" int cmve_eval_batch_finish(cmve_handle_t h, cmve_eval_batch_t b) {
  CMVE_REQUIRE(h && b && b->d_items, "cmve_eval_batch_finish: NULL handle / batch");
  CMVE_REQUIRE(b->pending && b->pending_stream == h->stream,
               "cmve_eval_batch_finish: the batch has no chained run awaiting its finish on this stream");
  if (CMVE_EVAL_FIX_CHAINED && b->chainable && b->fix_launch && b->c0.nb <= cmve::EVAL_FIXC_MAXB) {
    const int sf = cmve::launch_eval_batch(b->sq0, b->sg0, b->c0, b->d_items, b->count, b->qf, b->gf, 1, h->stream);
    if (sf) return sf;
  }
  const int st = cmve::launch_eval_batch(b->sq0, b->sg0, b->c0, b->d_items, b->count, b->qf, b->gf, 2, h->stream);
  if (st) return st;
  b->pending = false;
  return CMVE_OK;
}

extern "C" int cmve_eval_batch_destroy(cmve_eval_batch_t b) {
  if (!b) return CMVE_OK;
  (void)hipFree(b->d_items);
  (void)hipFree(b->d_args);
  delete b;
  return CMVE_OK;
}

// The graph form: the four launches of one cmve_eval_ranks call captured once (their kernel arguments --
// every pointer and size -- are baked in) and replayed with one hipGraphLaunch per evaluation: the host
// side of an evaluation drops from four kernel launches to one graph launch.
struct cmve_eval_graph {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
};

extern "C" int cmve_eval_graph_create(cmve_handle_t h, cmve_rows_t* q, cmve_rows_t* g, int32_t mode,
                                      const int64_t* row_off, const int32_t* row_idx, const int64_t* col_off,
                                      const int32_t* col_idx, void* ws, int64_t ws_bytes, int64_t cand_cap, int64_t* out,
                                      cmve_eval_graph_t* graph) {
  CMVE_REQUIRE(h && graph, "cmve_eval_graph_create: NULL handle / output");
  *graph = nullptr;
  CMVE_HIP(hipStreamBeginCapture(h->stream, hipStreamCaptureModeRelaxed));
  const int st = cmve_eval_ranks(h, q, g, mode, row_off, row_idx, col_off, col_idx, ws, ws_bytes, cand_cap, out,
                                 -1);  // (mode may carry CMVE_EVAL_PAIRED)
  hipGraph_t gr = nullptr;
  const hipError_t e = hipStreamEndCapture(h->stream, &gr);
  if (st) {  // (the argument check failed inside the capture: nothing was enqueued)
    if (gr) (void)hipGraphDestroy(gr);
    return st;
  }
  CMVE_HIP(e);
  auto* eg = new cmve_eval_graph;
  eg->graph = gr;
  const hipError_t ie = hipGraphInstantiate(&eg->exec, gr, nullptr, nullptr, 0);
  if (ie != hipSuccess) {
    (void)hipGraphDestroy(gr);
    delete eg;
    CMVE_HIP(ie);
  }
  *graph = eg;
  return CMVE_OK;
}

extern "C" int cmve_eval_graph_launch(cmve_handle_t h, cmve_eval_graph_t graph) {
  CMVE_REQUIRE(h && graph && graph->exec, "cmve_eval_graph_launch: NULL handle / graph");
  CMVE_HIP(hipGraphLaunch(graph->exec, h->stream));
  return CMVE_OK;
}

extern "C" int cmve_eval_graph_destroy(cmve_eval_graph_t graph) {
  if (!graph) return CMVE_OK;
  if (graph->exec) CMVE_HIP(hipGraphExecDestroy(graph->exec));
  if (graph->graph) CMVE_HIP(hipGraphDestroy(graph->graph));
  delete graph;
  return CMVE_OK;
}

extern "C" int cmve_eval_timing(cmve_handle_t h, int32_t slot, float* ms3) {
  CMVE_REQUIRE(h && ms3 && slot >= 0 && slot < CMVE_EVAL_TIMING_SLOTS, "cmve_eval_timing: bad argument");
  hipEvent_t* ev = h->eval_ev[slot];
  CMVE_REQUIRE(ev[0] && ev[3], "cmve_eval_timing: slot %d never recorded", slot);
  CMVE_HIP(hipEventSynchronize(ev[3]));
  for (int k = 0; k < 3; ++k) CMVE_HIP(hipEventElapsedTime(&ms3[k], ev[k], ev[k + 1]));
  return CMVE_OK;
}

extern "C" int cmve_eval_kernel_timing(cmve_handle_t h, int32_t slot, float* ms4) {
  CMVE_REQUIRE(h && ms4 && slot >= 0 && slot < CMVE_EVAL_TIMING_SLOTS, "cmve_eval_kernel_timing: bad argument");
  hipEvent_t* kev = h->eval_kev[slot];
  const bool chained = h->eval_chained[slot];  // (cmve_eval_batch_run_chained: the finish ran in the next run's prep)
  const int last = chained ? (h->eval_no_fix[slot] ? 3 : 5) : 7;
  CMVE_REQUIRE(kev[0] && kev[last], "cmve_eval_kernel_timing: slot %d never recorded", slot);
  CMVE_HIP(hipEventSynchronize(kev[last]));
  for (int k = 0; k < 4; ++k) {
    if ((k == 2 && h->eval_no_fix[slot]) || (k == 3 && chained)) {  // no fix-up launch (re-scored in the rank GEMM) /
      ms4[k] = 0.f;                                                  // the finish deferred to the next chained run
      continue;
    }
    CMVE_HIP(hipEventElapsedTime(&ms4[k], kev[2 * k], kev[2 * k + 1]));
  }
  return CMVE_OK;
}
