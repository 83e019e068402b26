"""The C ABI library builds for gfx950, loads, and exports every symbol include/cmve.h declares.

CPU-only: no kernel is launched here (host-only entry points only)."""
import ctypes as C
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cmve.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(cmve_\w+)\s*\(", src, re.M)))


def test_header_declares_the_hot_path():
    names = declared_functions()
    for must in ("cmve_pack_rows", "cmve_sim_store", "cmve_gt_thresholds", "cmve_rank_count",
                 "cmve_rank_from_matrix", "cmve_gt_positions_from_matrix", "cmve_topk", "cmve_gt_ranks",
                 "cmve_eval_ranks", "cmve_eval_workspace", "cmve_merge_topk"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from cmve import _lib
    for name in declared_functions():
        assert hasattr(_lib.lib, name), f"{name} declared in cmve.h but not exported"
    assert set(declared_functions()) <= set(_lib.exported_symbols())


def test_host_only_entry_points():
    from cmve import _lib
    assert _lib.lib.cmve_abi_version() == 21
    n_pad, d_pad = C.c_int64(), C.c_int64()
    assert _lib.lib.cmve_pack_size(1000, 1024, C.byref(n_pad), C.byref(d_pad)) == 0
    assert (n_pad.value, d_pad.value) == (1024, 1024)
    assert _lib.lib.cmve_pack_size(1, 100, C.byref(n_pad), C.byref(d_pad)) == 0
    assert (n_pad.value, d_pad.value) == (256, 128)
    assert _lib.lib.cmve_pack_size(-1, 100, C.byref(n_pad), C.byref(d_pad)) < 0
    assert b"pack_size" in _lib.lib.cmve_last_error()


def test_rows_struct_layout_matches_header():
    from cmve import _lib
    # 4 int64 + 2 ptr + ptr + 2 int32 + int64 + 4 ptr + double + 2 ptr
    assert C.sizeof(_lib.Rows) == 8 * 4 + 8 * 2 + 8 + 4 * 2 + 8 + 8 * 4 + 8 + 8 * 2


def test_gfx950_code_object_present():
    from cmve import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_topk_batch_workspace_sizes_the_sample():
    """cmve_topk_batch_workspace (host-only): the sample covers ~k * n_g / 128 gallery rows,
    rounded up to the 256-row pad, and the workspace holds its score block."""
    from cmve import _lib
    q, g = _lib.Rows(), _lib.Rows()
    q.n, q.n_pad, q.d, q.d_pad = 16384, 16384, 1024, 1024
    g.n, g.n_pad, g.d, g.d_pad = 131072, 131072, 1024, 1024
    ns, nf = C.c_int64(), C.c_int64()
    assert _lib.lib.cmve_topk_batch_workspace(C.byref(q), C.byref(g), 10, C.byref(ns), C.byref(nf)) == 0
    assert ns.value == 10240
    assert nf.value >= 16384 * 10240
    assert _lib.lib.cmve_topk_batch_workspace(C.byref(q), C.byref(g), 33, C.byref(ns), C.byref(nf)) < 0
    assert b"k must be" in _lib.lib.cmve_last_error()


def test_eval_workspace_layout_host_only():
    """cmve_eval_workspace (host-only): grows with the candidate capacity and both padded sets; a
    capacity too small for the bucket counters is refused by cmve_eval_ranks (checked on the GPU)."""
    from cmve import _lib
    q, g = _lib.Rows(), _lib.Rows()
    q.n, q.n_pad, q.d, q.d_pad = 1000, 1024, 1024, 1024
    g.n, g.n_pad, g.d, g.d_pad = 1000, 1024, 1024, 1024
    b1, b2 = C.c_int64(), C.c_int64()
    assert _lib.lib.cmve_eval_workspace(C.byref(q), C.byref(g), 1 << 16, C.byref(b1)) == 0
    assert _lib.lib.cmve_eval_workspace(C.byref(q), C.byref(g), 1 << 17, C.byref(b2)) == 0
    assert b2.value - b1.value == 8 << 16
    assert b1.value >= (8 << 16) + 2 * 1024 * (8 + 4 + 4 + 4)
    assert _lib.lib.cmve_eval_workspace(C.byref(q), C.byref(g), 0, C.byref(b1)) < 0
