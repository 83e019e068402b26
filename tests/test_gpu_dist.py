"""GPU tests of the sharded-gallery path in ONE process: several ShardedGallery shards of
one gallery (uneven, one empty), coordinated through cmve.dist's own code -- the encoded GT-score
MAX, the summed counts, cmve_gt_ranks, and the HIP k-way merge of the per-shard top-k runs
(cmve_merge_topk) -- against the unsharded oracle.  The collectives themselves are exercised by the
gloo tests (tests/test_dist_gloo.py) and by bench.py at N > 1."""
import numpy as np
import pytest

from oracle import retrieval as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def _problem(n_g=1500, n_q=400, d=96, seed=21):
    rng = np.random.default_rng(seed)
    gal = rng.standard_normal((n_g, d)).astype(np.float32)
    gts = [[int(x) for x in rng.choice(n_g, size=int(rng.integers(0, 3)), replace=False)] for _ in range(n_q)]
    gts[0], gts[1], gts[2] = [7], [7, n_g - 100], []  # a lone NaN GT, a NaN + finite list, no GT
    qs = (gal[[g[0] if g else 0 for g in gts]] + 1.2 * rng.standard_normal((n_q, d))).astype(np.float32)
    gal[[7, 40, n_g - 297]] = 0.0                     # zero videos: NaN columns
    return gal, qs, gts


def _expected_topk(s, k):
    return np.argsort(-s, axis=1, kind="stable")[:, :k]  # NaN scores last, ties by index


@pytest.mark.parametrize("cuts", [(0, 500, 1000, 1500), (0, 100, 1100, 1500), (0, 1500, 1500)])
def test_shards_in_process_match_unsharded_oracle(torch_cuda, cuts):
    torch = torch_cuda
    from cmve import engine, _lib, dist as D
    gal, qs, gts = _problem()
    n_g, n_q = gal.shape[0], qs.shape[0]
    with np.errstate(invalid="ignore", divide="ignore"):
        s = R.exact_scores64(qs, gal)
    shards = [D.ShardedGallery(gal[lo:hi], offset=lo, n_global=n_g) for lo, hi in zip(cuts[:-1], cuts[1:])]
    q = engine.RowSet(qs, with_lo=False)
    mode = _lib.SIM_F16
    keys = []
    for sh in shards:
        off, idx = sh.local_gt_csr(gts)
        sgt, _, _ = engine.gt_thresholds(q, sh.shard, off, idx, mode)
        keys.append(D.encode_gt_scores(sgt))
    sgt = D.decode_gt_scores(torch.stack(keys).max(dim=0).values)
    total = None
    for sh in shards:
        hi, lo = engine.rank_thresholds(q, sh.shard, sgt, mode)
        cnt, _ = engine.rank_count_launch(q, sh.shard, mode, row=(sgt, hi, lo), ws=sh.ws)
        assert not sh.ws.overflowed()
        total = cnt.clone() if total is None else total + cnt
    ranks = D.ranks_from(total, sgt, n_q, n_g).cpu().numpy()
    assert np.array_equal(ranks, R.rank_counts(s, gts))
    assert ranks[0] == n_g and ranks[2] == n_g + 1
    # top-k: each shard's exact local top-k with global ids, the runs side by side, the HIP merge
    k = 10
    runs_i, runs_s = [], []
    for sh in shards:
        kk = min(k, sh.shard.n)
        if kk < 1:
            i_g = torch.full((n_q, k), -1, dtype=torch.int64, device=q.device)
            s_g = torch.full((n_q, k), float("nan"), dtype=torch.float64, device=q.device)
        else:
            i_l, s_l = engine.topk(q, sh.shard, kk, mode=mode, to_host=False)
            i_g = torch.where(i_l >= 0, i_l.to(torch.int64) + sh.offset, i_l.to(torch.int64))
            i_g, s_g = D.pad_topk(i_g, s_l, k)
        runs_i.append(i_g)
        runs_s.append(s_g)
    top, top_s = D.merge_sorted_topk(torch.cat(runs_i, 1), torch.cat(runs_s, 1), len(shards), k)
    exp = _expected_topk(s, k)
    assert np.array_equal(top.cpu().numpy(), exp)
    np.testing.assert_allclose(top_s.cpu().numpy(), np.take_along_axis(s, exp, 1), rtol=0, atol=1e-13)


def test_sharded_gallery_world1_methods(torch_cuda):
    """ShardedGallery.rank_queries (overflow retry on a tiny list) and .topk at world 1, an empty shard's
    topk (all slots empty), and the merge kernel's ordering rules on hand-made runs."""
    torch = torch_cuda
    from cmve import engine, dist as D
    gal, qs, gts = _problem(n_g=800, n_q=256, seed=5)
    with np.errstate(invalid="ignore", divide="ignore"):
        s = R.exact_scores64(qs, gal)
    sh = D.ShardedGallery(gal, offset=0, n_global=gal.shape[0])
    sh.ws = engine.RankWorkspace(sh.device, cap=8)
    qt = torch.from_numpy(qs).cuda()
    ranks = sh.rank_queries(qt, sh.local_gt_csr(gts), qs.shape[0])
    assert sh.ws.cap > 8
    assert np.array_equal(ranks, R.rank_counts(s, gts))
    top, _ = sh.topk(qt, 7)
    assert np.array_equal(top, _expected_topk(s, 7))
    empty = D.ShardedGallery(gal[:0], offset=800, n_global=800)
    i_e, s_e = empty.topk(qt, 5)
    assert (i_e == -1).all() and np.isnan(s_e).all()
    # hand-made runs: ties by id, NaN after numbers, empty slots last, fewer entries than k
    ids = torch.tensor([[5, 2, 9, -1, 0, 1, 3, 4]], dtype=torch.int64, device="cuda")
    sc = torch.tensor([[0.9, 0.5, float("nan"), float("nan"), 0.5, 0.5, 0.1, float("nan")]], dtype=torch.float64,
                      device="cuda")
    o_i, o_s = D.merge_sorted_topk(ids, sc, 2, 8)
    assert o_i.tolist() == [[5, 0, 1, 2, 3, 4, 9, -1]]
    assert np.isnan(o_s.cpu().numpy()[0, 5:]).all()
