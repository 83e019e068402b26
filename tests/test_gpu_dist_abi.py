"""cmve_dist_* (the gallery-shard collectives in the C ABI, RCCL opened by dlopen) on one rank: a
single-rank communicator on its own stream; all-gather of the query rows is the identity, the MAX / SUM
reductions leave best-GT scores (incl. -inf "no GT here") and counts unchanged; calls without a
communicator fail with a message.  (N > 1 needs one GPU per rank: the driver's multi-GPU run exercises
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
        best = torch.tensor([0.25, -float("inf"), 0.5, -0.125], dtype=torch.float64, device=dev)
        counts = torch.tensor([3, 0, 7, 12], dtype=torch.int32, device=dev)
        b0, c0 = best.clone(), counts.clone()
        torch.cuda.synchronize()
        _lib.check(_lib.lib.cmve_dist_reduce_rank(h, engine._ptr(best), engine._ptr(counts), 4),
                   "cmve_dist_reduce_rank")
        st.synchronize()
        assert torch.equal(gathered, local)
        assert torch.equal(best, b0) and torch.equal(counts, c0)
        other = engine.stream_handle(dev, torch.cuda.Stream(dev))  # no communicator on this handle
        assert _lib.lib.cmve_dist_allgather_q(other, engine._ptr(local), 37, 64, engine._ptr(gathered)) != 0
        assert b"no communicator" in _lib.lib.cmve_last_error()
    finally:
        _lib.check(_lib.lib.cmve_dist_destroy(h), "cmve_dist_destroy")
