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


def test_sharded_gallery_over_c_abi_comm(torch_cuda):
    """ShardedGallery's two-direction evaluation, cal_perf and top-k driven through CAbiComm (the C ABI's RCCL
    communicator: cmve_dist_allreduce / cmve_dist_allgather / cmve_dist_size, run even at world 1) against the
    same calls over the default communicator and the oracle: identical ranks, tuples and top-k lists; the
    plain collectives reject unsupported dtypes."""
    import numpy as np
    import torch
    from cmve import _lib
    from cmve.dist import CAbiComm, ShardedGallery
    from oracle import retrieval as R
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(44)
    n, nq, d = 2500, 1800, 256
    v = rng.standard_normal((n, d)).astype(np.float32)
    gt = rng.integers(0, n, nq)
    c = (v[gt] + 1.3 * rng.standard_normal((nq, d))).astype(np.float32)
    t2v = [[int(g)] for g in gt]
    v2t = [[] for _ in range(n)]
    for i, g in enumerate(gt):
        v2t[int(g)].append(i)
    comm = CAbiComm(dev)
    try:
        assert (comm.rank, comm.world) == (0, 1)
        a = ShardedGallery(torch.from_numpy(v).to(dev), offset=0, n_global=n, device=dev, comm=comm)
        b = ShardedGallery(torch.from_numpy(v).to(dev), offset=0, n_global=n, device=dev)
        qt = torch.from_numpy(c).to(dev)
        ra, va = a.evaluate(qt, t2v, v2t)
        rb, vb = b.evaluate(qt, t2v, v2t)
        s = R.exact_scores64(c, v)
        assert np.array_equal(ra, rb) and np.array_equal(va, vb)
        assert np.array_equal(ra, R.rank_counts(s, t2v)) and np.array_equal(va, R.rank_counts(s.T, v2t))
        t2v_d = {i: l for i, l in enumerate(t2v)}
        assert a.cal_perf(qt, v2t, t2v_d) == b.cal_perf(qt, v2t, t2v_d)
        ia, sa = a.topk(qt, 10)
        ib, sb = b.topk(qt, 10)
        assert np.array_equal(ia, ib) and np.array_equal(sa, sb)
        with pytest.raises(ValueError):
            comm.all_reduce(torch.zeros(4, dtype=torch.int16, device=dev), "sum")
        x = torch.arange(6, dtype=torch.int64, device=dev)
        comm.all_reduce(x, "max")
        out = torch.empty(6, dtype=torch.int64, device=dev)
        comm.all_gather_into(out, x)
        torch.cuda.synchronize()
        assert x.tolist() == list(range(6)) and out.tolist() == list(range(6))
    finally:
        comm.close()
