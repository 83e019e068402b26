/*
 * cmve.h -- C ABI of libcmve.so, the MI355X-native (gfx950) retrieval hot path.
 *
 * The reference (WWWindrunner/Cross-Modal-Video-Engine) is pure Python/numpy;
 * it has no FFI.  Each entry point below replaces a Python/numpy call site on
 * the retrieval hot path; the replaced site is cited per function.  The Python
 * host mirror (cross-modal-video-engine_amd/cmve) binds these with ctypes and
 * keeps the reference's call signatures.
 *
 * Conventions
 *  - every call returns int status: 0 = CMVE_OK, negative = CMVE_E_*;
 *    cmve_last_error() returns a thread-local message for the last failure.
 *  - all array arguments are caller-owned DEVICE pointers (HBM), unless a
 *    parameter says "host".  No call allocates or synchronises: work is
 *    enqueued on the handle's stream (graph-capturable).
 *  - row-major matrices, leading dimension in ELEMENTS.
 */
#ifndef CMVE_H
#define CMVE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CMVE_ABI_VERSION 21

enum cmve_status {
  CMVE_OK = 0,
  CMVE_E_INVALID = -1,   /* bad argument / shape */
  CMVE_E_HIP = -2,       /* HIP runtime error (launch / memset) */
  CMVE_E_UNSUPPORTED = -3,
};

enum cmve_dtype { CMVE_F32 = 0, CMVE_F64 = 1, CMVE_BF16 = 2, CMVE_I32 = 3, CMVE_I64 = 4 };

/* precision of the similarity MFMA pass */
enum cmve_sim_mode {
  CMVE_SIM_BF16 = 0,    /* hi . hi                         (one bf16 MFMA per k-step)   */
  CMVE_SIM_BF16X3 = 1,  /* hi.hi + hi.lo + lo.hi  (split-bf16, ~1e-6 of fp64 cosine)     */
  CMVE_SIM_F16 = 2,     /* h16 . h16  fp16 plane, same MFMA rate as bf16, 8x finer rounding */
};

/* rank directions for cmve_rank_count */
enum cmve_rank_dir { CMVE_DIR_ROW = 1, CMVE_DIR_COL = 2 };

/* cmve_rows_t.flags */
#define CMVE_PACK_RAW 1   /* pack the rows as given (no L2 normalisation): GEMM operands of cmve_linear */

/* Tile geometry of the packed planes: rows padded to CMVE_ROW_ALIGN,
 * dimension padded to CMVE_DIM_ALIGN (zero fill). */
#define CMVE_ROW_ALIGN 256
#define CMVE_DIM_ALIGN 64

/*
 * A packed, L2-normalised embedding set resident in HBM.  Produced by
 * cmve_pack_rows; consumed by every scoring call.  All pointers are device
 * pointers owned by the caller (sizes from cmve_pack_size).
 *   hi/lo   : [n_pad, d_pad] bf16 planes; x_hat ~= hi (+ lo)
 *   raw     : the caller's un-normalised input rows (f32 or f64) -- read by
 *             the exact fp64 fix-up; must stay alive while the set is used
 *   inv_norm: [n_pad] fp64 1/||raw_i|| (NaN for a zero row when eps == 0)
 *   err_hi  : [n_pad] upper bound of ||x_hat_i - hi_i||_2
 *   err_hilo: [n_pad] upper bound of ||x_hat_i - hi_i - lo_i||_2
 *   h16     : [n_pad, d_pad] fp16 plane of x_hat (NULL if the set has no fp16 plane)
 *   err_h16 : [n_pad] upper bound of ||x_hat_i - h16_i||_2
 *   err_max : [3] max over rows of err_hi / err_hilo / err_h16
 */
typedef struct cmve_rows {
  int64_t n, d, n_pad, d_pad;
  uint16_t* hi;
  uint16_t* lo;
  const void* raw;
  int32_t raw_dtype;
  int32_t flags;         /* CMVE_PACK_* */
  int64_t raw_ld;
  double* inv_norm;
  float* err_hi;
  float* err_hilo;
  float* err_max;
  double eps;            /* normalisation epsilon: 0 = LINAS l2norm, 1e-12 = F.normalize */
  uint16_t* h16;
  float* err_h16;
} cmve_rows_t;

typedef struct cmve_handle* cmve_handle_t;

/* ---- handle / errors ---------------------------------------------------- */
int cmve_abi_version(void);
const char* cmve_last_error(void);
int cmve_create(int device, void* hip_stream, cmve_handle_t* out);
int cmve_set_stream(cmve_handle_t h, void* hip_stream);
int cmve_destroy(cmve_handle_t h);

/* Test hook: runs crafted v_mfma_f32_16x16x32_{bf16,f16} cases on one wave and writes
 * the 10 fp32 results (5 bf16 cases, 5 f16 cases) to out10 (device).  The rank error
 * bound's accumulation model is asserted against these (tests/test_gpu_numerics.py). */
int cmve_mfma_probe(cmve_handle_t h, float* out10);

/* padded sizes for a [n, d] set */
int cmve_pack_size(int64_t n, int64_t d, int64_t* n_pad, int64_t* d_pad);

/*
 * K1 -- row L2 normalisation + split-bf16 packing of an embedding set.
 * Replaces: LINAS-engine/evaluation.py:10-14 (l2norm), LINAS-engine/model.py:35-40
 * (l2norm, no eps), MultiFusion/src/combiner.py:134,180 and
 * MultiFusion/src/validate.py:55 (F.normalize, eps 1e-12).
 * Fills rows->{hi, lo, h16, inv_norm, err_hi, err_hilo, err_h16, err_max}; rows->raw/
 * raw_dtype/raw_ld/n/d/eps describe the input.  lo and h16 may be NULL (planes not
 * wanted); hi is always written.
 */
int cmve_pack_rows(cmve_handle_t h, cmve_rows_t* rows);

/*
 * K1' -- plain row normalisation y = x / max(||x||, eps)  (f32/f64 in, f32/f64 out).
 * Replaces the same sites as cmve_pack_rows when the caller wants the normalised
 * matrix itself (e.g. MultiFusion predicted features).
 */
int cmve_l2norm_rows(cmve_handle_t h, const void* x, int32_t x_dtype, int64_t ldx,
                     void* y, int32_t y_dtype, int64_t ldy, int64_t n, int64_t d, double eps);

/*
 * K4(a) -- similarity GEMM with store epilogue: out[i, j] = alpha * (q_i . g_j) + beta
 * for i < q->n, j < g->n.  bf16 / split-bf16 MFMA, LDS-staged 128x128x64 tiles.
 * Replaces: LINAS-engine/evaluation.py:21 (-1 * np.dot -> alpha=-1),
 * LINAS-engine/evaluation.py:83 (cal_simi, alpha=1), LINAS-engine/loss.py:10
 * (cosine_sim), MultiFusion/src/validate.py:73,90 and MultiFusion/src/inference.py:63
 * (1 - pred @ index.T -> alpha=-1, beta=1), MultiFusion/src/combiner.py:136 (alpha=100).
 * out_dtype: CMVE_F32 or CMVE_F64.
 */
int cmve_sim_store(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode,
                   float alpha, float beta, void* out, int32_t out_dtype, int64_t ldo);

/*
 * K3 -- projection GEMM with fused epilogue (MFC / Latent_mapping in eval mode,
 * LINAS-engine/model.py:97-116,374-381):  out[i, j] = BN( resid[i, j] + act( x_i . w_j + bias[j] ) )
 * with act (`relu` argument) 0 none, 1 ReLU, 2 QuickGELU x*sigmoid(1.702x), 3 sigmoid
 * (MultiFusion/src/combiner.py:7-9,105-106), resid optional (the fc2..fc4 residual layers, model.py:104-109),
 * BN eval as a per-column affine v * bn_scale + bn_shift (both NULL = no BN).  x [N, K] and
 * w [F_out, K] (torch nn.Linear layout) are packed with CMVE_PACK_RAW; mode CMVE_SIM_BF16X3
 * gives ~1e-6 relative error (the fp32 reference's own rounding is ~1e-7).  out fp32 [N, F_out].
 */
int cmve_linear(cmve_handle_t h, const cmve_rows_t* x, const cmve_rows_t* w, int32_t mode,
                const float* bias, const float* bn_scale, const float* bn_shift,
                const float* resid, int64_t ldr, int32_t relu, float* out, int64_t ldo);

/*
 * K2 -- temporal pooling.  collate: ragged frames [sum T_b, F] (row offsets[B+1]) ->
 * videos [B, t_max, F] (first min(max_len, T_b) frames, zero padded), origin [B, F] = mean
 * over ALL frames, mask [B, t_max] (LINAS-engine/util/tag_data_provider.py:91-109).
 */
int cmve_collate_frames(cmve_handle_t h, const float* frames, int64_t ldf, const int64_t* offsets,
                        int64_t B, int64_t F, int32_t max_len, int32_t t_max,
                        float* videos, float* origin, float* mask);

/* pool x[b, t, f] (strides in elements, f contiguous) over t -> out [B, F]:
 * mode 0 MEAN_VALID (t < lengths[b], LINAS-engine/model.py:152-156), 1 MEAN_ALL
 * (MultiFusion/src/combiner.py:140-143, MCT recognizer2d.py:76-83), 2 MAX_MASKED_ZERO
 * (max_t x*mask, masked steps contribute 0: model.py:157-158), 3 MAX_ALL (model.py:166). */
int cmve_temporal_pool(cmve_handle_t h, const float* x, int64_t stride_b, int64_t stride_t,
                       int64_t B, int64_t T, int64_t F, const int32_t* lengths, int32_t mode,
                       float* out, int64_t ldo);

/* K2 -- TSN feature-extraction head (MCT/mmaction/models/recognizers/recognizer2d.py:76-83, the
 * feature_extraction branch of Recognizer2D.forward_test): x = the backbone's maps [B * S, C, H, W]
 * (NCHW, contiguous; HW = H * W <= 128; HW = 1 for maps already pooled spatially, i.e. [B, S, C])
 * -> AdaptiveAvgPool2d(1) -> reshape (B, S, C) -> mean over the S segments -> out [B, C] (row
 * stride ldo).  fp32, plane sums in hw order.  B <= 65535 per call. */
int cmve_tsn_pool(cmve_handle_t h, const float* x, int64_t B, int64_t S, int64_t C, int64_t HW, float* out,
                  int64_t ldo);

/* K2 -- F.adaptive_avg_pool2d of the reference video's middle tokens before the single-query
 * combine (MultiFusion/src/inference.py:58-59: [1, T, 18*18, C] -> [1, T, 16, D]).
 * x: P planes of [H, W] fp32 (plane stride sp, row stride sh, columns contiguous);
 * out: [P, OH, OW] contiguous; ATen's windows [floor(i*H/OH), ceil((i+1)*H/OH)) per axis.
 * W <= 16384. */
int cmve_adaptive_avg_pool2d(cmve_handle_t h, const float* x, int64_t P, int64_t H, int64_t W,
                             int64_t sp, int64_t sh, int64_t OH, int64_t OW, float* out);

/*
 * K8/K9 -- non-GEMM pieces of MultiFusion Combiner.combine_features (MultiFusion/src/combiner.py:19-43,146-180):
 *   cmve_layernorm: y = LN(x) * gamma + beta (fp32 LayerNorm subclass, combiner.py:11-17)
 *   cmve_mha_1q: one query per batch element b (q [B, H*dh]) over T keys whose projected K/V rows
 *     are row t*B + b of kv (K at column 0, V at column v_off): the raw p_s_m.reshape(l*f, b, d)
 *     of combiner.py:164-165, which mixes batch rows -- reproduced, not fixed.  Scaled by dh^-0.5.
 *   cmve_fuse_combine: out = normalize(((y + ds*text) + (1-ds)*ref) + relu(based), eps)  (combiner.py:166,178-180)
 */
int cmve_layernorm(cmve_handle_t h, const float* x, int64_t ldx, int64_t n, int64_t d,
                   const float* gamma, const float* beta, double eps, float* y, int64_t ldy);
int cmve_mha_1q(cmve_handle_t h, const float* q, int64_t ldq, const float* kv, int64_t ldkv, int64_t v_off,
                int32_t B, int32_t T, int32_t H, int32_t dh, float* out, int64_t ldo);
int cmve_fuse_combine(cmve_handle_t h, const float* y, const float* ds, const float* text, const float* ref,
                      const float* based, int64_t n, int64_t d, double eps, float* out);
/* K9b: the same attention (combiner.py:38-40, k = v = p_s_m.reshape(l*f, b, d), combiner.py:159,164-166) with
 * the K / V in-projections absorbed: the host folds W_k into the query side, u [B, H*d] (per head
 * gamma (.) W_k,h^T q'_h / sqrt(dh), element order below), and W_v / out_proj into one GEMM after this call.
 * The key rows are read straight from the conv1x1 GEMM output y [B*f*npix, C] (row (bf, p), column c): key
 * t of query qb = g*gs + bb is run R % L of block bf = g*gs*f + R / L, R = t*gs + bb (cpr = d / npix channels
 * per run, L = C / cpr runs per block, T = f*L keys) -- the raw reshapes of combiner.py:159,164-165 for
 * B / gs consecutive batches of gs rows (gs = B: one batch).  Within a run, element e = p*cpr + c' is the
 * original element c'*npix + p.  Out: z [B, H*d] = per head sum_t softmax_t(u_h . n_t) n_t (n_t the
 * un-affined LayerNorm of key t, eps), in the kernel's element order; vmean [B, d] = v.mean(0) in the
 * original order.  Instantiated for (d, H) = (640, 8) and (512, 8). */
int cmve_mha_absorbed(cmve_handle_t h, const float* y, int64_t ldy, int64_t C, int64_t npix, int64_t f, int64_t gs,
                      int64_t B, int32_t H, int64_t d, const float* u, int64_t ldu, double eps, float* z, int64_t ldz,
                      float* vmean, int64_t ldv);
/*
 * The raw reshapes around Combiner's conv1x1 (MultiFusion/src/combiner.py:159,164): block b of x is
 * [R][C] row-major and its column c becomes row (b, c) of the output.
 *   cmve_transpose_blocks: fp32 out y [nb * C, R] (relu(conv(...)).reshape(b, f, l, -1) of the conv's
 *     [nb * 16, 640] output: R = 16, C = 640);
 *   cmve_pack_tblocks: out = the split-bf16 planes of the raw GEMM operand [nb * C, R] (the conv's
 *     input mid.reshape(b*f, 640, 16): R = 640, C = 16), written straight from x with no fp32
 *     transpose in between; out->{n, d, n_pad, d_pad} from cmve_pack_size, n_pad % C == 0;
 *   cmve_layernorm_pack: cmve_layernorm written as such planes (the K/V in-projection's operand).
 * The packed outputs carry CMVE_PACK_RAW (GEMM operands of cmve_linear only, err_max = +inf) and
 * hold bit for bit what cmve_pack_rows(CMVE_PACK_RAW) would make of the fp32 result.
 * R * (C + 1) * 4 <= 64 KiB; cmve_layernorm_pack: d <= 1024.
 */
int cmve_transpose_blocks(cmve_handle_t h, const float* x, int64_t nb, int64_t R, int64_t C, float* y);
int cmve_pack_tblocks(cmve_handle_t h, const float* x, int64_t nb, int64_t R, int64_t C, cmve_rows_t* out);
/* cmve_transpose_blocks with the attention's key order: the transposed output, read as rows of d
 * floats u = (g, t, bb) of p_s_m.reshape(G, T, gs, d), lands in row t*B + g*gs + bb (G = B / gs
 * consecutive batches of gs rows; gs = B is the reference's single-batch reshape(l*f, b, d),
 * combiner.py:164-165).  nb * R * C == B * T * d. */
int cmve_transpose_blocks_kv(cmve_handle_t h, const float* x, int64_t nb, int64_t R, int64_t C, int64_t d, int64_t T,
                             int64_t gs, int64_t B, float* y);
int cmve_layernorm_pack(cmve_handle_t h, const float* x, int64_t ldx, int64_t n, int64_t d, const float* gamma,
                        const float* beta, double eps, cmve_rows_t* out);

/*
 * K6 -- TripletLoss (LINAS-engine/loss.py:83-153) over a square score matrix S [B, B]
 * (S = im . s^T, rows = videos, columns = captions, cosine_sim loss.py:7-10).
 * dir bit 1 = cost_s (v2t, max over dim 1), bit 2 = cost_im (t2v, max over dim 0);
 * max_violation: hardest negative (first index on ties, as torch.max), else sum of all costs;
 * mean_style: cost_style 'mean'.  loss = device f32[1]; row_/col_ val/arg [B] are workspace
 * the backward reuses.  bwd writes dL/dS [B, B] for upstream gradient *g (device f32).
 */
int cmve_triplet_fwd(cmve_handle_t h, const float* S, int64_t ld, int32_t B, float margin,
                     int32_t max_violation, int32_t dir, int32_t mean_style, float* loss,
                     float* row_val, int32_t* row_arg, float* col_val, int32_t* col_arg);
int cmve_triplet_bwd(cmve_handle_t h, const float* S, int64_t ld, int32_t B, float margin,
                     int32_t max_violation, int32_t dir, int32_t mean_style, const float* g,
                     const int32_t* row_arg, const int32_t* col_arg, float* dS, int64_t ldd);

/*
 * K7 -- InfoNCE on logits scale * S: row half = CE(logits, arange) (MultiFusion/src/combiner_train.py:
 * 318,367-372), col half = CE(logits^T, arange) (MCT/mmaction/models/backbones/clip.py:383-386).
 * dir 1 row, 2 col, 3 both = (row + col) / 2.  loss3 (device f32[3]) = {row, col, selected};
 * row_lse/col_lse (f64 [B]) and row_loss/col_loss (f32 [B]) are workspace kept for the backward.
 */
int cmve_infonce_fwd(cmve_handle_t h, const float* S, int64_t ld, int32_t B, float scale, int32_t dir,
                     float* loss3, double* row_lse, double* col_lse, float* row_loss, float* col_loss);
int cmve_infonce_bwd(cmve_handle_t h, const float* S, int64_t ld, int32_t B, float scale, int32_t dir,
                     const float* g, const double* row_lse, const double* col_lse, float* dS, int64_t ldd);

/*
 * K15 -- element-pair losses of the distillation step (LINAS-engine/model.py:554-580 criteria,
 * :845-895 forward_loss_distill_similarity / forward_loss_distill):
 *   kind 0 MSE (x-y)^2, 1 SmoothL1 (beta 1), 2 KLDiv (input x, target y, log_target False:
 *   xlogy(y, y) - y*x, NaN for y < 0 as torch).  loss (device f32[1]) = scale * sum_i w_i f(x_i, y_i)
 *   (w nullable = 1; fp64 accumulation, one block: deterministic).  bwd: dx_i = g*scale*w_i*df/dx,
 *   dy_i = g*scale*w_i*df/dy (either output nullable), g = device f32[1] upstream gradient.
 */
int cmve_pair_loss_fwd(cmve_handle_t h, const float* x, const float* y, const float* w, int64_t n,
                       int32_t kind, float scale, float* loss);
int cmve_pair_loss_bwd(cmve_handle_t h, const float* x, const float* y, const float* w, int64_t n,
                       int32_t kind, float scale, const float* g, float* dx, float* dy);

/* fp32 GEMM for the loss gradient products and the training heads: C = alpha * op(A) . op(B) + beta * C
 * (op = transpose when trans* != 0; row-major) on v_mfma_f32_16x16x4_f32 -- each output is exactly a
 * k-ordered fp32 fmaf chain.  _ex adds bias[N] (nullable) and relu after the beta term. */
int cmve_gemm_f32(cmve_handle_t h, int32_t transA, int32_t transB, int64_t M, int64_t N, int64_t K,
                  float alpha, const float* A, int64_t lda, const float* B, int64_t ldb, float beta,
                  float* C, int64_t ldc);
int cmve_gemm_f32_ex(cmve_handle_t h, int32_t transA, int32_t transB, int64_t M, int64_t N, int64_t K,
                     float alpha, const float* A, int64_t lda, const float* B, int64_t ldb, float beta,
                     float* C, int64_t ldc, const float* bias, int32_t relu);

/*
 * K5a -- exact fp64 GT scores and rank thresholds for one direction.
 * For every row a of `a_set` with GT list idx[off[a] .. off[a+1]) into `b_set`:
 *   sgt[a]    = max_k cos64(a, b_k) over the GTs that score a number
 *               (NaN if the list is empty, +inf if every GT scores NaN -- a zero-norm row)
 *   thr_hi[a] = fp32 round-up  (sgt + E_a),  thr_lo[a] = fp32 round-down (sgt - E_a)
 * E_a is the rigorous error bound of the `mode` MFMA score.
 * Rows with no GT or padding get thr = +inf (never counted).  Arrays sized a_set->n_pad.
 * Replaces the GT lookup in LINAS-engine/util/metrics.py:140-147.
 */
int cmve_gt_thresholds(cmve_handle_t h, const cmve_rows_t* a_set, const cmve_rows_t* b_set,
                       int32_t mode, const int64_t* off, const int32_t* idx,
                       double* sgt, float* thr_hi, float* thr_lo);

/*
 * K4(b)+K5 -- fused score -> rank count, both directions in ONE GEMM pass, the
 * score matrix is never materialised:
 *   row_cnt[i] = #{ j : cos64(q_i, g_j) > row_sgt[i] }   (if CMVE_DIR_ROW in dirs)
 *   col_cnt[j] = #{ i : cos64(q_i, g_j) > col_sgt[j] }   (if CMVE_DIR_COL in dirs)
 * The MFMA pass counts the pairs that are certain under the error bound and
 * files the undecided (i, j) pairs in `cand` (capacity cand_cap, uint64 each;
 * its layout is internal to the library: per-bucket counters followed by buckets
 * of 256 gallery rows, so the fix-up reads each gallery row from HBM once);
 * an fp64 fix-up kernel re-scores those exactly.  *cand_count (device int64)
 * receives the number of undecided pairs; if it exceeds cand_cap the counts are
 * incomplete (a bucket overflowed) and the caller must retry with a buffer of at
 * least *cand_count entries.
 * gt rank (1-based) = 1 + cnt, i.e. the position of the best GT in the reference's
 * np.argsort (LINAS-engine/util/metrics.py:137-147) on tie-free inputs.
 * row_cnt/col_cnt are zeroed by the call.
 */
int cmve_rank_count(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode,
                    int32_t dirs,
                    const double* row_sgt, const float* row_hi, const float* row_lo,
                    const double* col_sgt, const float* col_hi, const float* col_lo,
                    int32_t* row_cnt, int32_t* col_cnt,
                    uint64_t* cand, int64_t cand_cap, int64_t* cand_count);

/* The two halves of cmve_rank_count, for callers that time or overlap them separately:
 * the MFMA pass (zeroes the counters, counts certain pairs, appends undecided ones) ... */
int cmve_rank_mfma(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, int32_t dirs,
                   const float* row_hi, const float* row_lo, const float* col_hi, const float* col_lo,
                   int32_t* row_cnt, int32_t* col_cnt, uint64_t* cand, int64_t cand_cap, int64_t* cand_count);
/* ... and the exact fp64 re-score of the undecided pairs. */
int cmve_rank_fixup(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t dirs,
                    const double* row_sgt, const double* col_sgt, int32_t* row_cnt, int32_t* col_cnt,
                    const uint64_t* cand, int64_t cand_cap, const int64_t* cand_count);
/*
 * cmve_rank_count with the fix-up hidden behind the MFMA pass: the gallery `g` is cut into
 * `chunks` row ranges (multiples of CMVE_ROW_ALIGN); chunk c's MFMA pass runs on the handle's
 * stream and its fp64 fix-up on an auxiliary stream of the handle as soon as that pass is done,
 * overlapping chunk c+1's MFMA pass.  Chunk c appends to cand[c*cap_c, (c+1)*cap_c) with
 * cap_c = cand_cap / chunks and counts into cand_count[c] (device int64[chunks]); if any
 * cand_count[c] > cap_c the counts are incomplete: retry with a larger cand_cap.  Results are
 * identical to cmve_rank_count.  Returns with all work ordered before later work on the handle's
 * stream.  1 <= chunks <= CMVE_MAX_CHUNKS.
 * Replaces: the single-stream argsort loop of LINAS-engine/util/metrics.py:137-147 (as cmve_rank_count).
 */
#define CMVE_MAX_CHUNKS 16
int cmve_rank_count_overlap(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode,
                            int32_t dirs,
                            const double* row_sgt, const float* row_hi, const float* row_lo,
                            const double* col_sgt, const float* col_hi, const float* col_lo,
                            int32_t* row_cnt, int32_t* col_cnt,
                            uint64_t* cand, int64_t cand_cap, int64_t* cand_count, int32_t chunks);
/* Summed duration of the MFMA passes of the handle's last cmve_rank_count_overlap (timing events
 * recorded on the handle's stream around each chunk's pass; waits for the last one) and the
 * number of passes: the per-launch duration a roofline figure needs while the fix-ups overlap. */
int cmve_overlap_mfma_ms(cmve_handle_t h, float* ms, int32_t* launches);

/*
 * Thresholds from GIVEN exact GT scores sgt[a_set->n] (NaN = no GT, +inf = every GT NaN): the sharded path,
 * where the owner rank of a query's GT computes sgt and all-gathers it with the query.
 * thr_hi/thr_lo as cmve_gt_thresholds, against the error bound of `b_set` (the local shard).
 */
int cmve_rank_thresholds(cmve_handle_t h, const cmve_rows_t* a_set, const cmve_rows_t* b_set, int32_t mode,
                         const double* sgt, float* thr_hi, float* thr_lo);

/*
 * 1-based GT ranks from the counts of cmve_rank_count and the GT scores of cmve_gt_thresholds
 * (LINAS-engine/util/metrics.py:137-147):
 *   ranks[i] = n_m + 1 if sgt[i] is NaN (empty GT list, metrics.py:140),
 *              n_m     if sgt[i] is +inf (every GT scores NaN: np.argsort puts NaN after every
 *                      finite score; numpy's order among several NaN is implementation-defined,
 *                      the GT is taken as the last),
 *              cnt[i] + 1 otherwise.
 * ranks (int64[n]) and/or recall (int64[4]: #rank<=1, #rank<=5, #rank<=10, sum of ranks,
 * metrics.py:149-157) may be NULL.
 */
int cmve_gt_ranks(cmve_handle_t h, const int32_t* cnt, const double* sgt, int64_t n, int64_t n_m,
                  int64_t* ranks, int64_t* recall);

/*
 * K14 -- one exact two-direction GT-rank evaluation of a resident problem in three or four launches
 * (the reference's per-validation chain LINAS-engine/validate.py:61-74 / tester.py:133-139:
 * evaluation.cal_error (evaluation.py:17-21) then util/metrics.eval_q2m t2v and v2t (metrics.py:124-157)).
 *   launch 1: pack q and g from their raw rows (as cmve_pack_rows), exact fp64 GT scores of both
 *             directions (as cmve_gt_thresholds), zeroed counters, err_max shards;
 *   launch 2: the fused rank GEMM (as cmve_rank_mfma), deriving the rank thresholds from the GT scores
 *             and the err_max shards in-kernel (a G256-sized problem gets them from one more small launch);
 *             each row's first GT pair is dropped from the undecided pairs (it is never counted); at G64
 *             size (fewer than 128 tiles of 128^2, e.g. MSR-VTT-1kA) the kernel re-scores its undecided pairs
 *             in fp64 itself (cmve_rank_fixup's arithmetic) and launch 3 is skipped;
 *   launch 3: the fp64 fix-up (as cmve_rank_fixup);
 *   launch 4: the ranks (as cmve_gt_ranks), R@K sums, the pair total and the sets' err_max.
 * The numbers equal the separate-launch path bit for bit.  q/g: packed sets (their planes, norms and
 * bounds are written; raw must point at the current rows).  row_off/row_idx: t2v GT lists of q's rows
 * into g (NULL: t2v off); col_off/col_idx: v2t GT lists of g's rows into q (NULL: v2t off).
 * ws: cmve_eval_workspace bytes, ZEROED ONCE when allocated (its err_max shards reset themselves).
 * out (int64, 16 + q->n + g->n): out[0..4) t2v #rank<=1, #<=5, #<=10, sum of ranks; out[4..8) the same
 * for v2t; out[8] undecided pairs; out[9] 0, or the cand_cap a retry needs (a bucket overflowed: the
 * ranks are incomplete); out[11] captions failing the CMVE_EVAL_PAIRED check; out[12] level-3 pairs; out[16 ..] t2v ranks, then v2t ranks (1-based; cmve_gt_ranks' rules).
 * timing_slot in [0, CMVE_EVAL_TIMING_SLOTS) records handle events around the launches
 * (cmve_eval_timing reads them) and each launch's own start / stop (cmve_eval_kernel_timing); -1 records none.
 * mode may carry CMVE_EVAL_PAIRED: the caller asserts a one-to-one GT pairing -- every t2v list is one
 * video p = row_idx[row_off[i]], every v2t list is one caption, and v2t(p) = [i] (MSR-VTT-1kA's
 * structure; q->n == g->n) -- and launch 1 then packs and scores each (caption, video) pair in one wave
 * (half the row reads; same results bit for bit).  Launch 1 checks the t2v side of the assertion per
 * caption (one GT, 0 <= p < g->n); a caption that fails it writes nothing of side g, ranks as if its list
 * were empty and is counted in out[11] (0 for a valid pairing): with out[11] != 0 the ranks are undefined,
 * but no write leaves the workspace / planes.  Lists whose v2t side is not the inverse (two captions naming
 * one video) give undefined ranks: both waves write that video's row (within bounds).
 * At F16 size with d_pad <= 1024 and 16-B aligned rows the workspace also holds a bf16 residual plane of
 * each side (x_hat - fp16 plane): launch 2 decides a band pair from fp16 + residual (error <= el_q +
 * (1 + el_q) el_g, ~7e-7) and lists the pairs within that bound (out[12] counts them; ~4 per 1k-A
 * evaluation), which the last launch re-scores in fp64 before it ranks (a full list: launch 2 re-scores the
 * rest itself).
 */
#define CMVE_EVAL_TIMING_SLOTS 32
#define CMVE_EVAL_PAIRED 0x100
#define CMVE_EVAL_OUT_HEAD 16
int cmve_eval_workspace(const cmve_rows_t* q, const cmve_rows_t* g, int64_t cand_cap, int64_t* bytes);
int cmve_eval_ranks(cmve_handle_t h, cmve_rows_t* q, cmve_rows_t* g, int32_t mode,
                    const int64_t* row_off, const int32_t* row_idx, const int64_t* col_off, const int32_t* col_idx,
                    void* ws, int64_t ws_bytes, int64_t cand_cap, int64_t* out, int32_t timing_slot);
/* Durations (ms) of the pack launch, the rank GEMM and the fix-up + ranks launches of the
 * cmve_eval_ranks call that used `slot` (waits for its last event). */
int cmve_eval_timing(cmve_handle_t h, int32_t slot, float* ms3);
/* the same evaluation's four kernel durations (ms4: prep, rank GEMM, fix-up, finish), each from its own
 * launch's start / stop (hipExtLaunchKernelGGL: the dispatch timestamps rocprofv3 reports, without the
 * dispatch gaps that events recorded between launches include; fix-up 0 when it ran inside the rank GEMM);
 * synchronises on the slot */
int cmve_eval_kernel_timing(cmve_handle_t h, int32_t slot, float* ms4);
/* Graph form of cmve_eval_ranks for an evaluation repeated on fixed buffers (the reference re-runs
 * validate.py:61-74 on new embeddings written into the same encode_* buffers; the bench's pipelined
 * steps): create captures the launches of one cmve_eval_ranks call (same arguments, no timing) on h's
 * stream into a HIP graph; every pointer and size is baked in, so q->raw / g->raw, the GT lists, ws and
 * out must stay at their addresses.  launch replays it on h's stream with one host call (same results
 * bit for bit); destroy frees it. */
/* K14 batches: `count` same-shaped evaluations (the same q / g sizes, dtypes, mode and GT lists; each its own
 * packed sets, workspace and output, as for cmve_eval_ranks) run as ONE prep, ONE rank GEMM and ONE finish
 * launch, each over (the blocks of one evaluation) x (the evaluations): a 1,000 x 1,000 evaluation's launches
 * leave most of the chip idle, a batch fills it.  The argument blocks are built and copied to the device at
 * create time (every pointer is baked in: refill the raw rows in place between runs, as for the graph form);
 * run enqueues the three launches on h's stream; the ranks and every R@K / overflow / pairing word equal
 * cmve_eval_ranks' (out[8] and out[12], the band-pair diagnostics, may differ by a few pairs: one evaluation's
 * G64 rank GEMM sums K in two halves, a batch's tile in one chain).  Batches take
 * the small-problem geometry (fewer than 128 tiles of 128^2, e.g. 1,000 x 1,000) with the rank GEMM's inline fp64
 * re-score (no overflow); the batch's rank GEMM runs 128 x 128 tiles (split-bf16: 128 x 64), each XCD taking a
 * contiguous run of the (evaluation, tile) pairs.
 * create synchronises (it uploads the table). */
typedef struct cmve_eval_batch* cmve_eval_batch_t;
int cmve_eval_batch_create(int32_t count, cmve_rows_t* const* q, cmve_rows_t* const* g, int32_t mode,
                           const int64_t* row_off, const int32_t* row_idx, const int64_t* col_off,
                           const int32_t* col_idx, void* const* ws, int64_t ws_bytes, int64_t cand_cap,
                           int64_t* const* out, cmve_eval_batch_t* batch);
/* timing_slot: -1, or a slot of h's timing ring receiving the batch's launch durations (cmve_eval_kernel_timing:
 * prep, rank GEMM, 0, finish; cmve_eval_timing: the event spans), as for cmve_eval_ranks */
int cmve_eval_batch_run(cmve_handle_t h, cmve_eval_batch_t batch, int32_t timing_slot);
/* Chained runs of a stream's successive batches (the headline's validation loop: LINAS-engine/validate.py:61-74 once
 * per evaluation): the run of `batch` defers its finish (ranks, R@K, pair total: the outputs' words) to the next
 * chained run on h's stream, whose first launch holds that finish beside its own prep (the specialised paired prep:
 * one launch; otherwise the finish runs as a launch of its own first).  prev: the batch chained on this stream
 * before (NULL: none); its outputs are complete once this call's first launch has run.  cmve_eval_batch_finish runs
 * a batch's deferred finish alone (after a stream's last chained run).  prev must have the batch's shapes and share
 * no workspace and no output range with it (refused otherwise: its finish adds into its outputs while this batch's
 * prep zeroes them).  Results equal cmve_eval_batch_run's bit for bit; timing_slot records the launches
 * (cmve_eval_timing: the prep span includes the previous finish; cmve_eval_kernel_timing: prep (the fused launch
 * with the previous finish, or the prep launch alone when the finish ran as a launch of its own), rank GEMM,
 * fix-up, 0).  A batch whose chained run
 * awaits its finish is refused by every run call until that finish is enqueued (as the prev of the next chained
 * run on the same stream, or by cmve_eval_batch_finish on it); prev must be such a batch of h's stream. */
int cmve_eval_batch_run_chained(cmve_handle_t h, cmve_eval_batch_t batch, cmve_eval_batch_t prev, int32_t timing_slot);
int cmve_eval_batch_finish(cmve_handle_t h, cmve_eval_batch_t batch);
int cmve_eval_batch_destroy(cmve_eval_batch_t batch);
typedef struct cmve_eval_graph* cmve_eval_graph_t;
int cmve_eval_graph_create(cmve_handle_t h, cmve_rows_t* q, cmve_rows_t* g, int32_t mode,
                           const int64_t* row_off, const int32_t* row_idx, const int64_t* col_off,
                           const int32_t* col_idx, void* ws, int64_t ws_bytes, int64_t cand_cap, int64_t* out,
                           cmve_eval_graph_t* graph);
int cmve_eval_graph_launch(cmve_handle_t h, cmve_eval_graph_t graph);
int cmve_eval_graph_destroy(cmve_eval_graph_t graph);

/*
 * Gallery-shard collectives over RCCL, for a C / C++ host that shards the
 * gallery without torch.distributed.  (The Python host mirror, cmve/dist.py, runs the same exchange
 * through torch.distributed -- backend "nccl" is RCCL -- and is the product path of bench.py; these
 * entry points are its twin for hosts without torch.)  Every rank holds a resident shard; per batch the
 * query rows are all-gathered, each rank scores its shard (cmve_gt_thresholds / cmve_rank_mfma +
 * cmve_rank_fixup / cmve_topk), the best-GT scores are all-reduced MAX and the better-than-GT counts SUM,
 * and the per-shard top-k runs are all-gathered and merged.  The reference never shards
 * (LINAS-engine/evaluation.py:17-21 and inference.py:78-79 score one in-memory gallery); these replace
 * nothing one-for-one.
 * RCCL (librccl.so) is opened with dlopen at first use (thread-safe).  cmve_dist_unique_id fills 128 bytes
 * on ONE rank; the host distributes them; cmve_dist_init binds a communicator of `nranks` to the handle
 * (its device, its stream for every collective; it makes the handle's device the calling thread's current
 * device); cmve_dist_destroy / cmve_destroy release it.
 * allgather_q: gathered[r * n_local + i] = rank r's local row i (n_local rows of d fp32 per rank).
 * reduce_rank: best_gt (fp64 [n], in place) in cmve_gt_thresholds' per-shard encoding -- NaN = no GT in
 *   this shard, +inf = GTs in this shard that all score NaN, else the best finite score -- becomes the
 *   global best-GT score in the same encoding (a finite score anywhere wins, then "all NaN", then "no GT":
 *   the kernel maps NaN -> -inf and +inf -> -1e300 before the MAX and back after it, so RCCL never sees a
 *   NaN); the result feeds cmve_rank_thresholds / cmve_gt_ranks unchanged.  counts (int32 [n], in place):
 *   SUM.  Either pointer may be NULL.
 * allgather_topk: every rank's exact local top-k (ids int64 [n_q, k] as GLOBAL gallery ids, -1 = empty
 *   slot; scores fp64 [n_q, k]; each row sorted score desc / id asc) is gathered into the caller's
 *   gathered_ids / gathered_scores (nranks * n_q * k each) and merged (as cmve_merge_topk) into
 *   out [n_q, k_out] on every rank.  nranks <= 64.
 */
#define CMVE_DIST_UNIQUE_ID_BYTES 128
int cmve_dist_unique_id(void* id);
int cmve_dist_init(cmve_handle_t h, int32_t nranks, int32_t rank, const void* id);
int cmve_dist_allgather_q(cmve_handle_t h, const float* local, int64_t n_local, int64_t d, float* gathered);
int cmve_dist_reduce_rank(cmve_handle_t h, double* best_gt, int32_t* counts, int64_t n);
int cmve_dist_allgather_topk(cmve_handle_t h, const int64_t* ids, const double* scores, int64_t n_q, int32_t k,
                             int64_t* gathered_ids, double* gathered_scores, int32_t k_out, int64_t* out_ids,
                             double* out_scores);
/* plain collectives on the handle's stream (dtype CMVE_F32 / F64 / I32 / I64): in-place all-reduce
 * (op CMVE_DIST_SUM / CMVE_DIST_MAX) of `count` elements, and all-gather of `count` elements per rank into
 * gathered[nranks * count] in rank order -- the two-direction exchange's int64 SUM (t2v counts, v2t R@K sums,
 * overflow flag) and the layout / v2t-rank gathers of cmve/dist.py's ShardedGallery over this communicator
 * (CAbiComm).  cmve_dist_size: the communicator's size and this handle's rank. */
#define CMVE_DIST_SUM 0
#define CMVE_DIST_MAX 1
int cmve_dist_allreduce(cmve_handle_t h, void* buf, int64_t count, int32_t dtype, int32_t op);
int cmve_dist_allgather(cmve_handle_t h, const void* local, int64_t count, int32_t dtype, void* gathered);
int cmve_dist_size(cmve_handle_t h, int32_t* nranks, int32_t* rank);
int cmve_dist_destroy(cmve_handle_t h);

/*
 * C3 -- k-way merge of per-shard exact top-k lists (the gallery sharded over ranks, SURVEY.md 8e;
 * the merge replaces the single-gallery np.argsort(errors[0])[:topK] of LINAS-engine/inference.py:79).
 * ids/scores: [n_q, lists * k_in] row-major (the all-gathered shard lists of each query side by side);
 * each run of k_in is sorted (score desc, id asc) with empty slots (id < 0) at its tail.
 * out: [n_q, k_out], score desc / global id asc, NaN scores after every number, empty slots id -1 /
 * score NaN.  1 <= lists <= 64.
 */
int cmve_merge_topk(cmve_handle_t h, const int64_t* ids, const double* scores, int64_t n_q, int32_t lists,
                    int32_t k_in, int32_t k_out, int64_t* out_ids, double* out_scores);

/*
 * Rank from a given score matrix (no GEMM): for each row i of errors[n_q, n_m]
 * (f32 or f64, lower = better, as LINAS errors), with GT lists off/idx:
 *   cnt[i] = #{ j : e_ij < min_{k in GT(i)} e_ik }   over the GTs that are not NaN
 *   (0 if GT(i) is empty: the caller maps empty lists to rank n_m + 1, as metrics.py:140
 *   initialises it; n_m - 1 if every GT is NaN, i.e. rank n_m as cmve_gt_ranks).
 * transposed != 0 ranks the columns of `errors` instead (errors.T rows).
 * Replaces: LINAS-engine/util/metrics.py:124-147 (eval_q2m's argsort loop).
 */
int cmve_rank_from_matrix(cmve_handle_t h, const void* errors, int32_t dtype, int64_t n_rows,
                          int64_t n_cols, int64_t ld, int32_t transposed,
                          const int64_t* off, const int32_t* idx, int32_t* cnt);

/*
 * Positions of every GT item in a given error matrix (mAP, LINAS-engine/util/metrics.py:61-102):
 *   pos[k] = #{ j : e_ij < e_{i, idx[k]} }   for every k in [off[i], off[i+1])
 * (position in np.argsort = pos + 1 on tie-free rows; a NaN GT gets n_cols / n_rows).
 * transposed != 0 ranks the columns of `errors` (errors.T rows).  pos is int32 [off[n]].
 */
int cmve_gt_positions_from_matrix(cmve_handle_t h, const void* errors, int32_t dtype, int64_t n_rows,
                                  int64_t n_cols, int64_t ld, int32_t transposed,
                                  const int64_t* off, const int32_t* idx, int32_t* pos);

/*
 * K4(c) -- exact top-k per query (LINAS-engine/inference.py:78-79:
 * np.argsort(errors[0])[:topK]).  Approximate scores s~ go to the workspace: for
 * q->n <= 32 a gallery-streaming MFMA GEMV (the inference.py regime: one caption
 * against the whole gallery, HBM-bound), else the MFMA GEMM.  A per-query
 * histogram of s~ bounds the k-th largest score T~_k from below; every column
 * within 2E of that bound (E = rigorous score error bound) is a candidate; one
 * block per query selects T~_k among the candidates, keeps the band
 * s~ >= T~_k - 2E (at most 4096 columns), re-scores it in fp64 and sorts it
 * (score desc, index asc).  out_idx [q->n, k] int32, out_score [q->n, k] fp64
 * (the exact cosine).  *overflow (device int32) becomes non-zero if a query's
 * band kept more than 4096 columns (retry with CMVE_SIM_BF16X3, whose band is
 * ~10x narrower).  1 <= k <= 2048.
 * scores_ws: device workspace of at least cmve_topk_workspace() floats
 * (ws_floats); its first q->n x g->n_pad floats hold s~ row-major.
 */
int cmve_topk_workspace(const cmve_rows_t* q, const cmve_rows_t* g, int32_t k, int64_t* n_floats);
int cmve_topk(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, int32_t k,
              float* scores_ws, int64_t ws_floats, int32_t* out_idx, double* out_score, int32_t* overflow);

/*
 * K13 -- exact top-k for a large query batch WITHOUT the n_q x n_g score matrix (the north
 * star's 16,384-caption batches against a gallery shard; same contract and results as
 * cmve_topk, LINAS-engine/inference.py:78-79 applied per caption).
 *   1. s~ of every query against the first `sample_rows` gallery rows (written by
 *      cmve_topk_batch_workspace): its per-query histogram gives tau_i <= T~_k(sample) - 2E
 *      <= T~_k(gallery) - 2E;
 *   2. one MFMA pass over the whole gallery whose epilogue emits every s~ >= tau_i;
 *   3. per query: select T~_k among its entries, re-score the 2E band in fp64, sort
 *      (score desc, index asc).
 * A query whose entries exceed 512, whose band exceeds 256, or whose sample holds fewer than k
 * finite scores is left UNRESOLVED: out_idx[i, :] = -2, and *unresolved (device int32) counts
 * them; the caller re-runs those rows through cmve_topk (the host mirror does).  1 <= k <= 32
 * (the sample is ~k/128 of the gallery; beyond a quarter the dense path is cheaper);
 * the gallery shard must hold < 2^24 rows.
 */
int cmve_topk_batch_workspace(const cmve_rows_t* q, const cmve_rows_t* g, int32_t k, int64_t* sample_rows,
                              int64_t* n_floats);
/* K12f: the exact dense top-k step of topk's band-overflow fallback (a query whose error band holds more
 * than the candidate cap: near-duplicate gallery rows; engine._topk_dense_exact scores gallery chunks in
 * fp64 with cmve_pairwise DOT).  Per row: the k best of [best_s / best_i (kb <= k entries, global ids) |
 * scores[row, 0..nc) with ids j0 + c] by (score desc, id asc) -- np.argsort's order of the errors, NaN
 * last (as -inf), -0.0 == +0.0 -- into out_s / out_i [n_rows, k] (ids -1 / -inf past the candidates).
 * The reference's inference.py:79-80 full argsort, for the rows the fast path cannot decide. */
int cmve_topk_dense_merge(cmve_handle_t h, const double* best_s, const int64_t* best_i, int64_t kb,
                          const double* scores, int64_t lds, int64_t n_rows, int64_t nc, int64_t j0, int32_t k,
                          double* out_s, int64_t* out_i);
int cmve_topk_batch(cmve_handle_t h, const cmve_rows_t* q, const cmve_rows_t* g, int32_t mode, int32_t k,
                    float* ws, int64_t ws_floats, int32_t* out_idx, double* out_score, int32_t* unresolved);

/* ---- non-cosine measures ---------------------------------
 * K10: out[i, j] = alpha * f(A_i, B_j) + beta over all pairs, fp64 accumulation.
 *   CMVE_PW_SQ_L2   sum (a-b)^2          CMVE_PW_L2      sqrt(sum (a-b)^2)
 *   CMVE_PW_L1      sum |a-b|            CMVE_PW_ORDER   sqrt(sum max(0, b-a)^2)
 *   CMVE_PW_JACCARD sum min(a,b) / sum max(a,b)
 *   CMVE_PW_DOT     sum a*b as a k-ordered fp64 fma chain (identical rows score identically: the
 *                   exact dense fallback of the top-k, LINAS-engine/inference.py:78-79)
 * Replaces: LINAS-engine/evaluation.py:22-35,56-71 (scipy cdist 'euclidean' / 'minkowski' p=1,
 * l1_norm / l2_norm = -f/D - 1, -jaccard) and LINAS-engine/loss.py:13-73 (order_sim = -ORDER,
 * euclidean_sim / L2_sim = -SQ_L2, L1_sim = -L1, L1_sim_norm = L1/D - 1, L2_sim_norm = SQ_L2/D - 1,
 * jaccard_sim).  A, B: f32/f64 rows (device); out f32/f64 [na, nb] (device). */
enum cmve_pw_metric { CMVE_PW_SQ_L2 = 0, CMVE_PW_L2 = 1, CMVE_PW_L1 = 2, CMVE_PW_ORDER = 3, CMVE_PW_JACCARD = 4,
                      CMVE_PW_DOT = 5 };
int cmve_pairwise(cmve_handle_t h, const void* A, int32_t a_dtype, int64_t lda, int64_t na, const void* B,
                  int32_t b_dtype, int64_t ldb, int64_t nb, int64_t d, int32_t metric, double alpha, double beta,
                  void* out, int32_t out_dtype, int64_t ldo);

/* ---- training step of the projection heads ---------------
 * K11: what LINAS-engine/model.py:984-1004 (train_emb, style 'GT') runs around the GEMMs (K3 forward,
 * cmve_gemm_f32 backward) and the losses (K6/K7).  Device pointers, fp32 rows; statistics in fp64.
 *   cmve_bn_train_fwd  BatchNorm1d training forward (model.py:83-85,111-112): batch mean / biased
 *                      variance normalise; running_mean/var (nullable) updated with momentum and the
 *                      unbiased variance; save_mean / save_invstd [d] kept for the backward.  n > 1.
 *   cmve_bn_train_bwd  dx, dgamma, dbeta (each nullable) from dy and x (batch statistics recomputed in fp64).
 *   cmve_col_sum       out[d] = column sums of x [n, d] (nn.Linear bias gradient).
 *   cmve_resid_relu    out = resid + relu(z)  (model.py:104-109); cmve_relu_grad: dz = dout * (z > 0).
 *   cmve_l2norm_bwd    gradient of y = x / ||x|| (model.py:35-40, no epsilon).
 *   cmve_dropout       y = keep ? x / (1 - p) : 0, keep = hash(seed, offset + i) >= p (splitmix64
 *                      finaliser; nn.Dropout semantics, NOT torch's random stream); mask (nullable)
 *                      = keep bytes; call_counter (device int64, nullable): offset += counter << 32, then
 *                      counter += 1 on the stream (graph-capturable); cmve_mask_scale applies a mask (the backward).
 * Multi-tensor calls take HOST arrays of n device pointers / sizes (launched 24 tensors at a time,
 * pointers passed by value); all arithmetic stays on the device (no host synchronisation):
 *   cmve_grad_norm_multi  total = ||all grads||_2 (fp64 sums, fixed order) and
 *                         coef = min(1, max_norm / (total + 1e-6)) (torch clip_grad_norm_, model.py:1000-1001);
 *                         coef / total_norm are device f32[1] (either nullable).
 *   cmve_scale_multi      x_i *= coef[0] (the clip itself).
 *   cmve_adam_multi       one torch.optim.Adam update per tensor (model.py:593; amsgrad off), steps[i] >= 1
 *                         (the tensor's step count after this update); grad_scale (device f32[1], nullable):
 *                         the clip coefficient, applied to and written back into the grads first;
 *                         dev_step (device int64, nullable): capturable mode -- incremented on the stream and
 *                         used as every tensor's step (steps may then be NULL). */
int cmve_bn_train_fwd(cmve_handle_t h, const float* x, int64_t ldx, int64_t n, int64_t d, const float* gamma,
                      const float* beta, double eps, double momentum, float* running_mean, float* running_var,
                      float* y, int64_t ldy, float* save_mean, float* save_invstd);
int cmve_bn_train_bwd(cmve_handle_t h, const float* dy, int64_t lddy, const float* x, int64_t ldx, int64_t n,
                      int64_t d, const float* gamma, double eps, float* dx, int64_t lddx, float* dgamma, float* dbeta);
int cmve_col_sum(cmve_handle_t h, const float* x, int64_t ldx, int64_t n, int64_t d, float* out);
int cmve_resid_relu(cmve_handle_t h, const float* z, const float* resid, int64_t n, float* out);
int cmve_relu_grad(cmve_handle_t h, const float* z, const float* dout, int64_t n, float* dz);
int cmve_l2norm_bwd(cmve_handle_t h, const float* x, int64_t ldx, const float* dy, int64_t lddy, int64_t n, int64_t d,
                    float* dx, int64_t lddx);
int cmve_dropout(cmve_handle_t h, const float* x, int64_t n, float p, uint64_t seed, uint64_t offset, float* y,
                 uint8_t* mask, int64_t* call_counter);
int cmve_mask_scale(cmve_handle_t h, const float* x, const uint8_t* mask, int64_t n, float scale, float* y);
int cmve_grad_norm_multi(cmve_handle_t h, int32_t n, float* const* grads, const int64_t* numels, double max_norm,
                         float* coef, float* total_norm);
int cmve_scale_multi(cmve_handle_t h, int32_t n, float* const* xs, const int64_t* numels, const float* coef);
int cmve_adam_multi(cmve_handle_t h, int32_t n, float* const* params, float* const* grads, float* const* exp_avgs,
                    float* const* exp_avg_sqs, const int64_t* numels, const int64_t* steps, double lr, double beta1,
                    double beta2, double eps, double weight_decay, const float* grad_scale, int64_t* dev_step);

/* ---- Combiner training step --------------------------------
 * K16: MultiFusion/src/combiner_train.py:341-381 (combiner.train(); logits = combiner(ref, text, target);
 * CE(logits, arange); backward; Adam) around cmve_gemm_f32(_ex) (Linear / 1x1 conv / in-projection
 * GEMMs), K7 (CE) and K11 (dropout, Adam):
 *   cmve_act_fwd / _bwd          kind 0 ReLU, 1 Sigmoid, 2 QuickGELU x*sigmoid(1.702x)
 *                                (MultiFusion/src/combiner.py:8-9,104-105,151-176); bwd takes the INPUT x.
 *   cmve_layernorm_train_fwd     LayerNorm rows (fp64 statistics), row mean / rstd saved (combiner.py:11-17)
 *   cmve_layernorm_bwd           dx (nullable), dgamma / dbeta (nullable) from x, dy and the saved statistics
 *   cmve_mha_1q_bwd              gradients of cmve_mha_1q (q, and K / V rows t*B + b of kv at columns 0 / v_off):
 *                                softmax recomputed; dkv must not alias kv (combiner.py:38-43,164-165)
 *   cmve_combine_train_fwd       out = ((y + ds*text) + (1-ds)*ref) + based, ds [B] (combiner.py:178-179)
 *   cmve_combine_train_bwd       dtext = g ds, dref = g (1-ds), dds = sum_j g (text - ref) (outputs nullable)
 *   cmve_pool_mean_bwd           dx[b, t, :] = dy[b, :] / T (time_process, combiner.py:140-143) */
int cmve_act_fwd(cmve_handle_t h, const float* x, int64_t n, int32_t kind, float* y);
int cmve_act_bwd(cmve_handle_t h, const float* x, const float* dy, int64_t n, int32_t kind, float* dx);
int cmve_layernorm_train_fwd(cmve_handle_t h, const float* x, int64_t ldx, int64_t n, int64_t d, const float* gamma,
                             const float* beta, double eps, float* y, int64_t ldy, float* save_mean, float* save_rstd);
int cmve_layernorm_bwd(cmve_handle_t h, const float* x, int64_t ldx, const float* dy, int64_t lddy, int64_t n,
                       int64_t d, const float* gamma, const float* save_mean, const float* save_rstd, float* dx,
                       int64_t lddx, float* dgamma, float* dbeta);
int cmve_mha_1q_bwd(cmve_handle_t h, const float* q, int64_t ldq, const float* kv, int64_t ldkv, int64_t v_off,
                    int32_t B, int32_t T, int32_t H, int32_t dh, const float* dout, int64_t lddo, float* dq,
                    int64_t lddq, float* dkv, int64_t lddkv);
int cmve_combine_train_fwd(cmve_handle_t h, const float* y, const float* ds, const float* text, const float* ref,
                           const float* based, int64_t B, int64_t d, float* out);
int cmve_combine_train_bwd(cmve_handle_t h, const float* g, const float* ds, const float* text, const float* ref,
                           int64_t B, int64_t d, float* dtext, float* dref, float* dds);
int cmve_pool_mean_bwd(cmve_handle_t h, const float* dy, int64_t B, int64_t T, int64_t F, float* dx);

/* ---- on-disk feature store -------------------------------
 * BigFile: feature.bin = n_rows x dim float32, row-major (LINAS-engine/basic/bigfile.py:6-18).
 * These are HOST calls (they read the page cache); the device variant also enqueues H2D copies on
 * the handle's stream and waits only for its own staging halves.
 * Replaces: BigFile.read / read_one (LINAS-engine/basic/bigfile.py:23-60), called once per
 * frame by VisDataSet4DualEncoding.__getitem__ (LINAS-engine/util/tag_data_provider.py:330-337). */
typedef struct cmve_bigfile* cmve_bigfile_t;
/* map feature.bin read-only (validates its size against n_rows x dim) */
int cmve_bigfile_open(const char* feature_bin, int64_t n_rows, int32_t dim, cmve_bigfile_t* out);
int cmve_bigfile_close(cmve_bigfile_t bf);
/* out[k, :] = row rows[k] (host arrays; `threads` memcpy workers); a row outside [0, n_rows) is an error */
int cmve_bigfile_gather(cmve_bigfile_t bf, const int64_t* rows, int64_t n, float* out, int32_t threads);
/* dst[k, :] (device) = row rows[k], streamed through `staging` (pinned host, staging_rows x dim
 * floats, used as two halves: the H2D copy of one half overlaps the gather of the other).  staging
 * must stay untouched until the handle's stream has passed this call. */
int cmve_bigfile_gather_device(cmve_handle_t h, cmve_bigfile_t bf, const int64_t* rows, int64_t n, float* dst,
                               float* staging, int64_t staging_rows, int32_t threads);

#ifdef __cplusplus
}
#endif
#endif /* CMVE_H */
