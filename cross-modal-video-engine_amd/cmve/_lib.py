"""ctypes binding of libcmve.so (the C ABI declared in include/cmve.h).

The library is REQUIRED: importing this module without a built libcmve.so raises
ImportError -- there is no CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CMVE_LIB", os.path.join(_HERE, "libcmve.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(f"libcmve.so not found at {LIB_PATH}: build it with `make -C cross-modal-video-engine_amd` "
                      "(or __graft_entry__.build()); cmve has no CPU fallback")

lib = C.CDLL(LIB_PATH)

# ---- enums (include/cmve.h) ----
CMVE_OK = 0
CMVE_F32, CMVE_F64, CMVE_BF16, CMVE_I32, CMVE_I64 = 0, 1, 2, 3, 4
SIM_BF16, SIM_BF16X3, SIM_F16 = 0, 1, 2
DIR_ROW, DIR_COL = 1, 2
ROW_ALIGN, DIM_ALIGN = 256, 64
TOPK_MAX = 2048
MAX_CHUNKS = 16
EVAL_TIMING_SLOTS = 32
EVAL_OUT_HEAD = 16
EVAL_PAIRED = 0x100  # CMVE_EVAL_PAIRED
DIST_UNIQUE_ID_BYTES = 128  # CMVE_DIST_UNIQUE_ID_BYTES
DIST_SUM, DIST_MAX = 0, 1  # CMVE_DIST_SUM / CMVE_DIST_MAX
PACK_RAW = 1
POOL_MEAN_VALID, POOL_MEAN_ALL, POOL_MAX_MASKED_ZERO, POOL_MAX_ALL = 0, 1, 2, 3
PW_SQ_L2, PW_L2, PW_L1, PW_ORDER, PW_JACCARD, PW_DOT = 0, 1, 2, 3, 4, 5
PAIR_MSE, PAIR_SMOOTH_L1, PAIR_KL = 0, 1, 2
ACT_RELU_K, ACT_SIGMOID_K, ACT_QUICKGELU_K = 0, 1, 2


class Rows(C.Structure):
    """``cmve_rows_t`` -- a packed embedding set (device pointers)."""
    _fields_ = [
        ("n", C.c_int64), ("d", C.c_int64), ("n_pad", C.c_int64), ("d_pad", C.c_int64),
        ("hi", C.c_void_p), ("lo", C.c_void_p),
        ("raw", C.c_void_p), ("raw_dtype", C.c_int32), ("flags", C.c_int32), ("raw_ld", C.c_int64),
        ("inv_norm", C.c_void_p), ("err_hi", C.c_void_p), ("err_hilo", C.c_void_p), ("err_max", C.c_void_p),
        ("eps", C.c_double),
        ("h16", C.c_void_p), ("err_h16", C.c_void_p),
    ]


_vp, _i32, _i64, _f32, _f64 = C.c_void_p, C.c_int32, C.c_int64, C.c_float, C.c_double
_P = C.POINTER

SIGNATURES = {
    "cmve_abi_version": (C.c_int, []),
    "cmve_last_error": (C.c_char_p, []),
    "cmve_create": (C.c_int, [C.c_int, _vp, _P(_vp)]),
    "cmve_set_stream": (C.c_int, [_vp, _vp]),
    "cmve_destroy": (C.c_int, [_vp]),
    "cmve_mfma_probe": (C.c_int, [_vp, _vp]),
    "cmve_pack_size": (C.c_int, [_i64, _i64, _P(_i64), _P(_i64)]),
    "cmve_pack_rows": (C.c_int, [_vp, _P(Rows)]),
    "cmve_l2norm_rows": (C.c_int, [_vp, _vp, _i32, _i64, _vp, _i32, _i64, _i64, _i64, _f64]),
    "cmve_sim_store": (C.c_int, [_vp, _P(Rows), _P(Rows), _i32, _f32, _f32, _vp, _i32, _i64]),
    "cmve_linear": (C.c_int, [_vp, _P(Rows), _P(Rows), _i32, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _i64]),
    "cmve_collate_frames": (C.c_int, [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp]),
    "cmve_temporal_pool": (C.c_int, [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _vp, _i32, _vp, _i64]),
    "cmve_pair_loss_fwd": (C.c_int, [_vp, _vp, _vp, _vp, _i64, _i32, C.c_float, _vp]),
    "cmve_pair_loss_bwd": (C.c_int, [_vp, _vp, _vp, _vp, _i64, _i32, C.c_float, _vp, _vp, _vp]),
    "cmve_act_fwd": (C.c_int, [_vp, _vp, _i64, _i32, _vp]),
    "cmve_act_bwd": (C.c_int, [_vp, _vp, _vp, _i64, _i32, _vp]),
    "cmve_layernorm_train_fwd": (C.c_int, [_vp, _vp, _i64, _i64, _i64, _vp, _vp, C.c_double, _vp, _i64, _vp, _vp]),
    "cmve_layernorm_bwd": (C.c_int, [_vp, _vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    "cmve_mha_1q_bwd": (C.c_int, [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _vp, _i64, _vp, _i64,
                                  _vp, _i64]),
    "cmve_combine_train_fwd": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp]),
    "cmve_combine_train_bwd": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp, _vp]),
    "cmve_pool_mean_bwd": (C.c_int, [_vp, _vp, _i64, _i64, _i64, _vp]),
    "cmve_tsn_pool": (C.c_int, [_vp, _vp, _i64, _i64, _i64, _i64, _vp, _i64]),
    "cmve_adaptive_avg_pool2d": (C.c_int, [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _vp]),
    "cmve_layernorm": (C.c_int, [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _f64, _vp, _i64]),
    "cmve_mha_1q": (C.c_int, [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _vp, _i64]),
    "cmve_eval_batch_create": (C.c_int, [C.c_int32, _vp, _vp, C.c_int32, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp,
                                         _vp]),
    "cmve_eval_batch_run": (C.c_int, [_vp, _vp, C.c_int32]),
    "cmve_eval_batch_run_chained": (C.c_int, [_vp, _vp, _vp, C.c_int32]),
    "cmve_eval_batch_finish": (C.c_int, [_vp, _vp]),
    "cmve_eval_batch_destroy": (C.c_int, [_vp]),
    "cmve_topk_dense_merge": (C.c_int, [_vp, _vp, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _i32, _vp, _vp]),
    "cmve_mha_absorbed": (C.c_int, [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i64, _vp, _i64, _f64,
                                    _vp, _i64, _vp, _i64]),
    "cmve_fuse_combine": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _f64, _vp]),
    "cmve_triplet_fwd": (C.c_int, [_vp, _vp, _i64, _i32, _f32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
    "cmve_triplet_bwd": (C.c_int, [_vp, _vp, _i64, _i32, _f32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _i64]),
    "cmve_infonce_fwd": (C.c_int, [_vp, _vp, _i64, _i32, _f32, _i32, _vp, _vp, _vp, _vp, _vp]),
    "cmve_infonce_bwd": (C.c_int, [_vp, _vp, _i64, _i32, _f32, _i32, _vp, _vp, _vp, _vp, _i64]),
    "cmve_gemm_f32": (C.c_int, [_vp, _i32, _i32, _i64, _i64, _i64, _f32, _vp, _i64, _vp, _i64, _f32, _vp, _i64]),
    "cmve_gt_thresholds": (C.c_int, [_vp, _P(Rows), _P(Rows), _i32, _vp, _vp, _vp, _vp, _vp]),
    "cmve_rank_count": (C.c_int, [_vp, _P(Rows), _P(Rows), _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                  _vp, _i64, _vp]),
    "cmve_rank_mfma": (C.c_int, [_vp, _P(Rows), _P(Rows), _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64,
                                 _vp]),
    "cmve_rank_fixup": (C.c_int, [_vp, _P(Rows), _P(Rows), _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "cmve_rank_count_overlap": (C.c_int, [_vp, _P(Rows), _P(Rows), _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                          _vp, _vp, _i64, _vp, _i32]),
    "cmve_overlap_mfma_ms": (C.c_int, [_vp, _P(_f32), _P(_i32)]),
    "cmve_rank_thresholds": (C.c_int, [_vp, _P(Rows), _P(Rows), _i32, _vp, _vp, _vp]),
    "cmve_gt_ranks": (C.c_int, [_vp, _vp, _vp, _i64, _i64, _vp, _vp]),
    "cmve_eval_workspace": (C.c_int, [_P(Rows), _P(Rows), _i64, _P(_i64)]),
    "cmve_eval_ranks": (C.c_int, [_vp, _P(Rows), _P(Rows), _i32, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _i32]),
    "cmve_eval_timing": (C.c_int, [_vp, _i32, _P(_f32)]),
    "cmve_eval_kernel_timing": (C.c_int, [_vp, _i32, _P(_f32)]),
    "cmve_eval_graph_create": (C.c_int, [_vp, _P(Rows), _P(Rows), _i32, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp,
                                         _P(_vp)]),
    "cmve_eval_graph_launch": (C.c_int, [_vp, _vp]),
    "cmve_eval_graph_destroy": (C.c_int, [_vp]),
    "cmve_dist_unique_id": (C.c_int, [_vp]),
    "cmve_dist_init": (C.c_int, [_vp, _i32, _i32, _vp]),
    "cmve_dist_allgather_q": (C.c_int, [_vp, _vp, _i64, _i64, _vp]),
    "cmve_dist_reduce_rank": (C.c_int, [_vp, _vp, _vp, _i64]),
    "cmve_dist_allgather_topk": (C.c_int, [_vp, _vp, _vp, _i64, _i32, _vp, _vp, _i32, _vp, _vp]),
    "cmve_dist_allreduce": (C.c_int, [_vp, _vp, _i64, _i32, _i32]),
    "cmve_dist_allgather": (C.c_int, [_vp, _vp, _i64, _i32, _vp]),
    "cmve_dist_size": (C.c_int, [_vp, _vp, _vp]),
    "cmve_dist_destroy": (C.c_int, [_vp]),
    "cmve_merge_topk": (C.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _i32, _vp, _vp]),
    "cmve_rank_from_matrix": (C.c_int, [_vp, _vp, _i32, _i64, _i64, _i64, _i32, _vp, _vp, _vp]),
    "cmve_gt_positions_from_matrix": (C.c_int, [_vp, _vp, _i32, _i64, _i64, _i64, _i32, _vp, _vp, _vp]),
    "cmve_topk_workspace": (C.c_int, [_P(Rows), _P(Rows), _i32, _P(_i64)]),
    "cmve_topk": (C.c_int, [_vp, _P(Rows), _P(Rows), _i32, _i32, _vp, _i64, _vp, _vp, _vp]),
    "cmve_topk_batch_workspace": (C.c_int, [_P(Rows), _P(Rows), _i32, _P(_i64), _P(_i64)]),
    "cmve_topk_batch": (C.c_int, [_vp, _P(Rows), _P(Rows), _i32, _i32, _vp, _i64, _vp, _vp, _vp]),
    "cmve_transpose_blocks": (C.c_int, [_vp, _vp, _i64, _i64, _i64, _vp]),
    "cmve_pack_tblocks": (C.c_int, [_vp, _vp, _i64, _i64, _i64, _P(Rows)]),
    "cmve_transpose_blocks_kv": (C.c_int, [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _vp]),
    "cmve_layernorm_pack": (C.c_int, [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _f64, _P(Rows)]),
    "cmve_pairwise": (C.c_int, [_vp, _vp, _i32, _i64, _i64, _vp, _i32, _i64, _i64, _i64, _i32, _f64, _f64, _vp,
                                _i32, _i64]),
    "cmve_bn_train_fwd": (C.c_int, [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _f64, _f64, _vp, _vp, _vp, _i64, _vp, _vp]),
    "cmve_bn_train_bwd": (C.c_int, [_vp, _vp, _i64, _vp, _i64, _i64, _i64, _vp, _f64, _vp, _i64, _vp, _vp]),
    "cmve_gemm_f32_ex": (C.c_int, [_vp, _i32, _i32, _i64, _i64, _i64, _f32, _vp, _i64, _vp, _i64, _f32, _vp, _i64,
                                   _vp, _i32]),
    "cmve_col_sum": (C.c_int, [_vp, _vp, _i64, _i64, _i64, _vp]),
    "cmve_resid_relu": (C.c_int, [_vp, _vp, _vp, _i64, _vp]),
    "cmve_relu_grad": (C.c_int, [_vp, _vp, _vp, _i64, _vp]),
    "cmve_l2norm_bwd": (C.c_int, [_vp, _vp, _i64, _vp, _i64, _i64, _i64, _vp, _i64]),
    "cmve_dropout": (C.c_int, [_vp, _vp, _i64, C.c_float, C.c_uint64, C.c_uint64, _vp, _vp, _vp]),
    "cmve_mask_scale": (C.c_int, [_vp, _vp, _vp, _i64, C.c_float, _vp]),
    "cmve_grad_norm_multi": (C.c_int, [_vp, _i32, _vp, _vp, _f64, _vp, _vp]),
    "cmve_scale_multi": (C.c_int, [_vp, _i32, _vp, _vp, _vp]),
    "cmve_adam_multi": (C.c_int, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _f64, _f64, _f64, _f64, _f64, _vp,
                                  _vp]),
    "cmve_bigfile_open": (C.c_int, [C.c_char_p, _i64, _i32, _P(_vp)]),
    "cmve_bigfile_close": (C.c_int, [_vp]),
    "cmve_bigfile_gather": (C.c_int, [_vp, _vp, _i64, _vp, _i32]),
    "cmve_bigfile_gather_device": (C.c_int, [_vp, _vp, _vp, _i64, _vp, _vp, _i64, _i32]),
}

for _name, (_res, _args) in SIGNATURES.items():
    _fn = getattr(lib, _name)  # AttributeError here = a declared symbol is not exported
    _fn.restype = _res
    _fn.argtypes = _args

ABI_VERSION = 21
if lib.cmve_abi_version() != ABI_VERSION:
    raise ImportError(f"libcmve.so ABI version {lib.cmve_abi_version()} != {ABI_VERSION}: rebuild it")


class CmveError(RuntimeError):
    pass


def check(status, what=""):
    if status != CMVE_OK:
        msg = lib.cmve_last_error().decode(errors="replace")
        raise CmveError(f"{what or 'cmve call'} failed with status {status}: {msg}")


def exported_symbols():
    return sorted(SIGNATURES)
