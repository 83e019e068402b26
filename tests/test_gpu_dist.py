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


# ---- the two-direction sharded evaluation (cal_perf over N shards), LocalGroup: one thread + HIP stream per shard ----

def test_local_group_evaluate_and_cal_perf_match_oracle(torch_cuda):
    """ShardedGallery.evaluate / cal_perf over 3 and 4 in-process shards (uneven caption slices, an empty
    last shard, NaN columns, several captions per video): t2v and v2t ranks and the reference's cal_perf
    tuples (mAP included) equal the unsharded oracle."""
    torch = torch_cuda
    from cmve import dist as D
    rng = np.random.default_rng(33)
    n_q, d = 60, 64
    for n_g in (9, 700):
        gal = rng.standard_normal((n_g, d)).astype(np.float32)
        owner = rng.integers(0, n_g, n_q)
        zero = [j for j in range(2, n_g, 13) if j not in set(owner.tolist())]
        gal[zero] = 0.0  # zero videos without captions: NaN columns, empty v2t lists
        qs = (gal[owner] + 0.9 * rng.standard_normal((n_q, d))).astype(np.float32)
        v2t, t2v = R.get_gt([f"v{j}" for j in range(n_g)], [f"v{int(o)}#{i}" for i, o in enumerate(owner)])
        t2v_lists = [t2v[i] for i in range(n_q)]
        with np.errstate(invalid="ignore", divide="ignore"):
            s = R.exact_scores64(qs, gal)
            exp_perf = R.cal_perf(-s, v2t, t2v)
        for world in (3, 4):
            cuts = np.linspace(0, n_q, world + 1).astype(int)

            def body(r, comm):
                lo, hi = D.shard_bounds(n_g, world, r)
                sh = D.ShardedGallery(gal[lo:hi], offset=lo, n_global=n_g, comm=comm)
                q_local = torch.from_numpy(qs[cuts[r]:cuts[r + 1]]).cuda()
                return sh.evaluate(q_local, t2v_lists, v2t), sh.cal_perf(q_local, v2t, t2v)

            for (r_t, r_v), perf in D.LocalGroup(world).run(body):
                assert np.array_equal(r_t, R.rank_counts(s, t2v_lists))
                assert np.array_equal(r_v, R.rank_counts(s.T, v2t))
                for got, exp in zip(perf, exp_perf):
                    np.testing.assert_allclose(np.asarray(got, float), np.asarray(exp, float), rtol=0, atol=1e-12)


@pytest.fixture(scope="module")
def c3_unsharded(torch_cuda):
    """BASELINE configs[2] data (seed 2, 20,000 x 20,000 x 1024, sigma 10, one GT per caption),
    its unsharded K14 ranks (RankSession, both directions) and an independent fp64 check of them."""
    torch = torch_cuda
    from cmve import engine
    rng = np.random.default_rng(2)
    n, d = 20000, 1024
    v = rng.standard_normal((n, d), dtype=np.float32)
    c = (v + np.float32(10.0) * rng.standard_normal((n, d), dtype=np.float32)).astype(np.float32)
    gts = [[i] for i in range(n)]
    sess = engine.RankSession(n, n, d, row_gts=gts, col_gts=gts, dtype=torch.float32)
    t2v, v2t = sess.run(torch.from_numpy(c).cuda(), torch.from_numpy(v).cuda())
    ct = torch.from_numpy(c).cuda().double()
    vt = torch.from_numpy(v).cuda().double()
    ct = ct / ct.norm(dim=1, keepdim=True)
    vt = vt / vt.norm(dim=1, keepdim=True)
    exp_r = np.empty(n, np.int64)
    exp_c = np.zeros(n, np.int64)
    diag = (ct * vt).sum(dim=1)
    for b in range(0, n, 2000):
        s = ct[b:b + 2000] @ vt.T
        rows = torch.arange(s.shape[0], device=s.device)
        s[rows, rows + b] = -float("inf")
        exp_r[b:b + 2000] = 1 + (s > diag[b:b + 2000, None]).sum(dim=1).cpu().numpy()
        exp_c += (s > diag[None, :]).sum(dim=0).cpu().numpy()
    exp_c += 1
    del ct, vt, s
    torch.cuda.empty_cache()
    assert np.array_equal(t2v, exp_r) and np.array_equal(v2t, exp_c)  # K14 == independent fp64
    return v, c, gts, t2v, v2t


@pytest.mark.parametrize("world", [2, 4, 8])
def test_c3_sharded_both_directions_equal_unsharded(c3_unsharded, world):
    """The C3 gallery over `world` in-process shards (each its own thread + HIP stream; the same
    coordination code as RCCL ranks): every caption's t2v rank and every video's v2t rank equal the
    unsharded K14 evaluation (and so the fp64 check), and the v2t R@K sums carried by the counts'
    all-reduce equal the gathered ranks'."""
    import torch
    from cmve import dist as D
    v, c, gts, t2v, v2t = c3_unsharded
    n = v.shape[0]

    def body(r, comm):
        lo, hi = D.shard_bounds(n, world, r)
        sh = D.ShardedGallery(v[lo:hi], offset=lo, n_global=n, comm=comm)
        q_local = torch.from_numpy(c[lo:hi]).cuda()  # each rank holds its slice of the captions
        r_t, r_v = sh.evaluate(q_local, gts, gts)
        q_all = D.all_gather_var(q_local, comm)
        _, v_loc, rec, ovf = sh.evaluate_device(q_all, sh.local_gt_csr(gts), sh.local_v2t_csr(gts), n)
        return r_t, r_v, v_loc.cpu().numpy(), rec.tolist(), bool(ovf), (lo, hi)

    for r_t, r_v, v_loc, rec, ovf, (lo, hi) in D.LocalGroup(world).run(body):
        assert np.array_equal(r_t, t2v), int((r_t != t2v).sum())
        assert np.array_equal(r_v, v2t), int((r_v != v2t).sum())
        assert np.array_equal(v_loc, v2t[lo:hi]) and not ovf
        assert rec == [int((v2t <= 1).sum()), int((v2t <= 5).sum()), int((v2t <= 10).sum()), int(v2t.sum())]
