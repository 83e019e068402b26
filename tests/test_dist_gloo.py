"""world_size-2 gloo rehearsal of the sharded-gallery protocol on CPU.

Each rank scores its contiguous gallery shard with the ORACLE (the GPU kernels are covered
by the -m gpu tests); everything else is the product coordination code of cmve.dist:
all-gather of queries, all-reduce(MAX) of per-shard GT scores, all-reduce(SUM) of counts,
global ranks, and the gathered top-k merge.  Results must equal the unsharded oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import retrieval as R


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_g, n_q, d, k, q_per_rank, result_q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "cross-modal-video-engine_amd"))
    sys.path.insert(0, os.path.dirname(here))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cmve import dist as D  # coordination helpers only (no GPU needed)
        rng = np.random.default_rng(11)
        gal = rng.standard_normal((n_g, d))
        gts = [list(rng.choice(n_g, size=int(rng.integers(0, 3)), replace=False)) for _ in range(n_q)]
        used = {int(x) for g in gts for x in g}
        zero = [j for j in range(3, n_g, 7) if j not in used]
        gal[zero] = 0.0  # zero videos (never a GT): NaN scores, ranked last in index order
        qs = gal[[g[0] if g else 0 for g in gts]] + 0.8 * rng.standard_normal((n_q, d))
        lo, hi = D.shard_bounds(n_g, world, rank)
        # each rank contributes its query slice; all-gather restores the global order
        q_local = torch.from_numpy(qs[rank * q_per_rank:(rank + 1) * q_per_rank].copy())
        q_all = torch.empty((world * q_per_rank, d), dtype=q_local.dtype)
        work = D.gather_rows_async(q_local, q_all, world)  # the bench's overlapped form
        work.wait()
        assert np.array_equal(q_all.numpy(), qs)
        assert bool(D.any_flag(torch.tensor(rank == 1), world)) and not bool(D.any_flag(torch.tensor(False), world))
        s = R.exact_scores64(q_all.numpy(), gal[lo:hi])             # local shard scores (oracle)
        local = D.local_gt_lists(gts, lo, hi)
        sgt = torch.tensor([s[i, l].max() if l else np.nan for i, l in enumerate(local)], dtype=torch.float64)
        sgt = D.merge_gt_scores(sgt, world)
        cnt = torch.tensor([int(np.count_nonzero(s[i] > sgt[i].item())) if not np.isnan(sgt[i].item()) else 0
                            for i in range(n_q)], dtype=torch.int32)
        cnt = D.reduce_counts(cnt, world)
        ranks_t = D.ranks_from(cnt, sgt, n_q, n_g)
        ranks = ranks_t.numpy()
        rc = D.recall_counts_device(ranks_t).tolist()
        assert rc == [int((ranks <= 1).sum()), int((ranks <= 5).sum()), int((ranks <= 10).sum()), int(ranks.sum())]
        kk = min(k, hi - lo)
        order = np.argsort(-s, axis=1, kind="stable")[:, :kk]
        idx_g = torch.from_numpy(order + lo)
        sc = torch.from_numpy(np.take_along_axis(s, order, axis=1))
        idx_g, sc = D.pad_topk(idx_g, sc, k)
        top, _ = D.merge_topk(idx_g, sc, k, world)
        if rank == 0:
            s_full = R.exact_scores64(qs, gal)
            exp_ranks = R.rank_counts(s_full, gts)
            exp_top = np.argsort(-s_full, axis=1, kind="stable")[:, :k]
            result_q.put((bool(np.array_equal(ranks, exp_ranks)), bool(np.array_equal(top, exp_top))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_g", [9, 301, 512])
def test_sharded_protocol_world2(n_g):
    world, n_q, d, k = 2, 40, 24, 7
    ctx = mp.get_context("spawn")
    result_q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_g, n_q, d, k, n_q // world, result_q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ranks_ok, top_ok = result_q.get()
    assert ranks_ok and top_ok


def test_merge_topk_single_shard_is_identity():
    """world 1: the shard's own top-k (already score desc, id asc) comes back unchanged; padded
    empty slots read -1 / NaN."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "cross-modal-video-engine_amd"))
    from cmve import dist as D
    idx = torch.tensor([[5, 2, 9], [1, 0, 3]])
    sc = torch.tensor([[0.9, 0.5, -float("inf")], [0.7, 0.7, 0.1]], dtype=torch.float64)
    idx, sc = D.pad_topk(idx, sc, 4)
    top, s = D.merge_topk(idx, sc, 4, 1)
    assert top.tolist() == [[5, 2, 9, -1], [1, 0, 3, -1]]
    assert np.isnan(s[:, 3]).all() and s[0, 2] == -np.inf
