// K14 evaluation (eval.hip): the argument blocks shared by its kernels and the host entry (sim.hip).
#pragma once
#include "cmve_internal.h"

namespace cmve {

constexpr int EVAL_ARRIVAL_WORDS = 9 * 64;  // workspace words zeroed at allocation: the err_max shards
constexpr int EMAX_SHARDS = EVAL_EMAX_SHARDS;  // per side and plane: [side][plane][shard] float bits

// one side of the problem: a packed set and the GT lists of the direction whose queries are its rows
struct EvalSide {
  const void* raw;
  int64_t ld;
  int64_t n, n_pad;
  int vec;  // fp32 rows, d % 4 == 0, 16-B aligned: float4 runs (pack_rows_kernel's VEC path)
  int flags;
  double eps;
  uint16_t* hi;
  uint16_t* lo;
  uint16_t* h16;
  double* inv;
  float* err_hi;
  float* err_hilo;
  float* err_h16;
  float* err_max;
  const int64_t* off;  // GT lists into the OTHER set; nullptr: this direction is off
  const int32_t* idx;
  double* sgt;
  float* thr_hi;
  float* thr_lo;
  int32_t* cnt;
  int64_t* ranks;      // out: 1-based ranks of this direction
  int32_t* gt1;        // the first GT of each row (idx[off[row]], -1: none / padding), written by the prep: the
                       // rank GEMM drops that GT pair from the undecided list (it can never be counted)
  uint16_t* lo16;      // F16 rank path: [n_pad, d_pad] bf16 residual plane of x_hat - h16 (lo16_elem), nullptr: off
  float* err_lo16;     // [n_pad] upper bound of ||x_hat - (h16 + lo16)||_2 (the level-2 re-score's bound)
};

struct EvalCommon {
  int64_t d, d_pad;
  int mode;
  unsigned* emax;              // err_max shards [2][3][EMAX_SHARDS] (float bits; zero at allocation, re-zeroed
                               // by every evaluation's finish)
  unsigned long long* bucket;  // bucket counters at the head of the undecided-pair buffer
  int64_t nb, cap_b;
  const uint64_t* cand;
  int64_t* stats;              // out[0, 16)
  int fix_inline;              // the rank GEMM re-scored the undecided pairs itself (no list: never an overflow)
  // level 3 (the fp64 re-score of the pairs the rank GEMM's level 2 left undecided) is deferred to the finish:
  // the GEMM appends (row | col << 31 | dirs << 62) to this list (count zeroed by the prep; a full list makes
  // the GEMM re-score inline instead), the finish's rank blocks re-score the entries of their rows / columns
  unsigned* l3_count;
  uint64_t* l3;
  int l3_cap;
  int dbg;                     // kernel studies only (CMVE_EVAL_DBG): skip parts, results garbage
  unsigned long long* stamps;  // kernel studies only (CMVE_EVAL_DBG & 128): [kernel][block][8] s_memrealtime
                               // (kernel 0 prep, 1 finish, 2 fix-up, 3 the rank GEMM's tiles)
};

// phase 0: pack + GT scores, phase 1: fix-up, phase 2: err_max + ranks + R@K (the rank GEMM runs between
// phases 0 and 1, sim.hip); stamp k of block b in kernel kern (0 prep, 1 finish, 2 fix-up) when stamps are on
#define EVAL_STAMP(cp, kern, k)                                                                                  \
  if ((cp).stamps && threadIdx.x == 0 && blockIdx.x < 1024)                                                     \
  (cp).stamps[((size_t)(kern) * 1024 + blockIdx.x) * 8 + (k)] = __builtin_amdgcn_s_memrealtime()
int launch_eval(const EvalSide& q, const EvalSide& g, const EvalCommon& c, int q_f64, int g_f64, int phase,
                hipStream_t s);
// one evaluation's argument blocks in a batch's device table (cmve_eval_batch_*)
struct EvalItem {
  EvalSide q, g;
  EvalCommon c;
};
#ifndef CMVE_EVAL_FIX_CHAINED
#define CMVE_EVAL_FIX_CHAINED 0  // study (with CMVE_EVAL_INLINE_L2=0): a batch's fix-up rides in the next chained launch
#endif
constexpr int64_t EVAL_FIXC_MAXB = 1024;  // the chained fix-up role's LDS bucket prefix (a 1k-A evaluation: 256)
// (xtab: a batch whose fix-up runs as a third role of the launch -- the CMVE_EVAL_FIX_CHAINED study only)
int launch_eval_batch_chained(const EvalSide& q, const EvalSide& g, const EvalCommon& c0, const EvalItem* ptab,
                              const EvalItem* ftab, int count, int q_f64, int g_f64, hipStream_t s,
                              const EvalItem* xtab = nullptr);
bool eval_batch_chainable(const EvalSide& q, const EvalSide& g, const EvalCommon& c0);
int launch_eval_batch(const EvalSide& q, const EvalSide& g, const EvalCommon& c0, const EvalItem* tab, int count,
                      int q_f64, int g_f64, int phase, hipStream_t s);

}  // namespace cmve
