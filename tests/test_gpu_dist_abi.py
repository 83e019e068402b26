"""cmve_dist_* (the gallery-shard collectives in the C ABI, RCCL opened by dlopen) on one rank: a
single-rank communicator on its own stream; all-gather of the query rows is the identity, the MAX / SUM
reductions leave best-GT scores in cmve_gt_thresholds' encoding (NaN "no GT here", +inf "every GT scores
NaN": encoded around the MAX inside the call) and counts unchanged; the top-k gather + merge returns the
rank's own sorted runs; calls without a communicator fail with a message.  (N > 1 needs one GPU per rank: the driver's multi-GPU run exercises
the torch.distributed path of cmve/dist.py, the same exchange.)"""
import ctypes

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def test_dist_c_abi_single_rank(torch_cuda):
    import torch
    from cmve import engine, _lib
    dev = torch.device("cuda", 0)
    uid = ctypes.create_string_buffer(_lib.DIST_UNIQUE_ID_BYTES)
    _lib.check(_lib.lib.cmve_dist_unique_id(uid), "cmve_dist_unique_id")
    st = torch.cuda.Stream(dev)
    h = engine.stream_handle(dev, st)
    _lib.check(_lib.lib.cmve_dist_init(h, 1, 0, uid), "cmve_dist_init")
    try:
        assert _lib.lib.cmve_dist_init(h, 1, 0, uid) != 0  # one communicator per handle
        local = torch.randn((37, 64), device=dev)
        gathered = torch.full_like(local, float("nan"))
        torch.cuda.synchronize()
        _lib.check(_lib.lib.cmve_dist_allgather_q(h, engine._ptr(local), 37, 64, engine._ptr(gathered)),
                   "cmve_dist_allgather_q")
        best = torch.tensor([0.25, float("nan"), float("inf"), -0.125], dtype=torch.float64, device=dev)
        counts = torch.tensor([3, 0, 7, 12], dtype=torch.int32, device=dev)
        b0, c0 = best.clone(), counts.clone()
        torch.cuda.synchronize()
        _lib.check(_lib.lib.cmve_dist_reduce_rank(h, engine._ptr(best), engine._ptr(counts), 4),
                   "cmve_dist_reduce_rank")
        st.synchronize()
        assert torch.equal(gathered, local)
        assert bool(((best == b0) | (best.isnan() & b0.isnan())).all())  # NaN / +inf survive the encoded MAX
        assert torch.equal(counts, c0)
        # top-k runs (global ids, fp64 scores, score desc / id asc, -1 empty slots at the tail)
        ids = torch.tensor([[9, 2, 4, -1], [1, 3, 5, 7]], dtype=torch.int64, device=dev)
        sc = torch.tensor([[0.9, 0.5, 0.5, float("nan")], [0.8, 0.7, 0.1, float("nan")]], dtype=torch.float64,
                          device=dev)
        g_i, g_s = torch.empty_like(ids), torch.empty_like(sc)
        o_i = torch.full((2, 3), -7, dtype=torch.int64, device=dev)
        o_s = torch.empty((2, 3), dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        _lib.check(_lib.lib.cmve_dist_allgather_topk(h, engine._ptr(ids), engine._ptr(sc), 2, 4, engine._ptr(g_i),
                                                     engine._ptr(g_s), 3, engine._ptr(o_i), engine._ptr(o_s)),
                   "cmve_dist_allgather_topk")
        st.synchronize()
        assert o_i.tolist() == [[9, 2, 4], [1, 3, 5]]
        assert o_s.tolist() == [[0.9, 0.5, 0.5], [0.8, 0.7, 0.1]]
        other = engine.stream_handle(dev, torch.cuda.Stream(dev))  # no communicator on this handle
        assert _lib.lib.cmve_dist_allgather_q(other, engine._ptr(local), 37, 64, engine._ptr(gathered)) != 0
        assert b"no communicator" in _lib.lib.cmve_last_error()
    finally:
        _lib.check(_lib.lib.cmve_dist_destroy(h), "cmve_dist_destroy")
