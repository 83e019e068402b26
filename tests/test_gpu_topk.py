"""GPU parity of the exact top-k path (inference.py scorer, LINAS-engine/inference.py:78-79) --
the small-batch MFMA GEMV (n_q <= 32), the histogram threshold, the candidate list and its
dense-row fallback -- against the fp64 oracle.  Bar: top-k ids bit-exact against a stable
argsort of the fp64 cosines (score desc, index asc; NaN columns last), scores to 1e-13.
"""
import os

import numpy as np
import pytest

from oracle import retrieval as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def _expect(s, k):
    order = np.argsort(-s, axis=1, kind="stable")[:, :k]
    return order, np.take_along_axis(s, order, axis=1)


def _check(idx, sc, s, k):
    order, best = _expect(s, k)
    assert idx.shape == order.shape
    for i in range(s.shape[0]):
        assert list(idx[i]) == list(order[i]), f"query {i}"
    fin = np.isfinite(best)
    np.testing.assert_allclose(sc[fin], best[fin], rtol=0, atol=1e-13)


@pytest.mark.parametrize("mode_name", ["SIM_F16", "SIM_BF16", "SIM_BF16X3"])
@pytest.mark.parametrize("nq,ng,d", [(1, 1, 64), (1, 5000, 1024), (7, 3000, 100), (16, 40000, 256),
                                     (17, 777, 640), (32, 20000, 1024), (33, 5000, 128)])
def test_topk_small_batch(torch_cuda, mode_name, nq, ng, d):
    """n_q <= 32 takes the gallery-streaming GEMV (one and two query tiles); 33 the GEMM."""
    from cmve import engine, _lib
    rng = np.random.default_rng(nq * 1000 + ng + d)
    gal = rng.standard_normal((ng, d)).astype(np.float32)
    qs = (gal[rng.integers(0, ng, nq)] + 3.0 * rng.standard_normal((nq, d))).astype(np.float32)
    s = R.exact_scores64(qs, gal)
    q = engine.RowSet(qs, with_lo=True)
    g = engine.RowSet(gal, with_lo=True)
    k = min(10, ng)
    idx, sc = engine.topk(q, g, k, mode=getattr(_lib, mode_name))
    _check(idx, sc, s, k)


@pytest.mark.parametrize("k", [1, 64, 2048])
def test_topk_large_gallery_one_query(torch_cuda, k):
    """inference.py's shape: one caption against a 262,144-video gallery (many histogram chunks)."""
    from cmve import engine
    rng = np.random.default_rng(5 + k)
    ng, d = 262144, 1024
    gal = rng.standard_normal((ng, d), dtype=np.float32)
    qs = (gal[[12345]] + 10.0 * rng.standard_normal((1, d))).astype(np.float32)
    s = (gal.astype(np.float64) @ qs[0].astype(np.float64)) / (
        np.linalg.norm(gal.astype(np.float64), axis=1) * np.linalg.norm(qs[0].astype(np.float64)))
    q = engine.RowSet(qs, with_lo=True)
    g = engine.RowSet(gal, with_lo=True)
    idx, sc = engine.topk(q, g, k)
    _check(idx, sc, s[None, :], k)


def test_topk_nan_rows_and_k_beyond_finite(torch_cuda):
    """Zero gallery rows (LINAS l2norm has no epsilon -> NaN scores) sort last, in index order; with
    fewer finite scores than k every column is kept."""
    from cmve import engine
    rng = np.random.default_rng(3)
    d = 96
    for ng, zeros, nq, k in [(8, [1, 4, 6, 7, 0], 3, 6), (3000, list(range(0, 3000, 7)), 20, 25),
                             (600, list(range(590)), 40, 12)]:
        gal = rng.standard_normal((ng, d))
        gal[zeros] = 0.0
        qs = rng.standard_normal((nq, d))
        s = R.exact_scores64(qs, gal)
        q = engine.RowSet(qs, eps=0.0, with_lo=True)
        g = engine.RowSet(gal, eps=0.0, with_lo=True)
        idx, sc = engine.topk(q, g, k)
        _check(idx, sc, s, k)


def test_topk_near_duplicates(torch_cuda):
    """A dense cluster of near-duplicate videos around the best match: many candidates share the
    histogram bins of the k-th score; ids stay exact."""
    from cmve import engine
    rng = np.random.default_rng(21)
    d = 512
    base = rng.standard_normal(d)
    gal = rng.standard_normal((30000, d))
    gal[:3000] = base + 0.02 * rng.standard_normal((3000, d))
    qs = base[None, :] + 0.5 * rng.standard_normal((4, d))
    s = R.exact_scores64(qs, gal)
    q = engine.RowSet(qs, with_lo=True)
    g = engine.RowSet(gal, with_lo=True)
    idx, sc = engine.topk(q, g, 50)
    _check(idx, sc, s, 50)


def test_topk_band_overflow_falls_back_to_exact(torch_cuda):
    """More than TOPK_CAP (4096) gallery rows tie at the k-th score (exact duplicates) and no lo plane
    for the split-bf16 retry: the dense fp64 fallback keeps the ids exact (ties by index)."""
    from cmve import engine
    rng = np.random.default_rng(22)
    d = 256
    gal = rng.standard_normal((20000, d))
    base = rng.standard_normal(d)
    dup = rng.choice(20000, 6000, replace=False)
    gal[dup] = base
    qs = np.stack([base + 0.3 * rng.standard_normal(d), rng.standard_normal(d)])
    s = R.exact_scores64(qs, gal)
    q = engine.RowSet(qs, with_lo=False)
    g = engine.RowSet(gal, with_lo=False)
    idx, sc = engine.topk(q, g, 10)
    _check(idx, sc, s, 10)
    assert set(idx[0]) <= set(dup.tolist())


def test_gallery_scorer_ids(torch_cuda):
    """inference.py mirror: GalleryScorer.topk_ids == [video_ids[i] for i in argsort(cal_error)[:topK]]."""
    from cmve.linas.inference import GalleryScorer
    rng = np.random.default_rng(2)
    gal = rng.standard_normal((4000, 128))
    ids = [f"video{i}" for i in range(4000)]
    cap = gal[[77]] + 0.8 * rng.standard_normal((1, 128)).astype(np.float32)
    sc = GalleryScorer(gal, ids)
    errors = R.cal_error(gal, cap)
    expect = [ids[i] for i in np.argsort(errors[0], kind="stable")[:10]]
    assert sc.topk_ids(cap, 10) == expect


# ---- K13: large-batch top-k without the score matrix (cmve_topk_batch) ----

def _batch_case(seed, nq, ng, d, sigma=3.0, dtype=np.float32):
    rng = np.random.default_rng(seed)
    gal = rng.standard_normal((ng, d)).astype(dtype)
    qs = (gal[rng.integers(0, ng, nq)] + sigma * rng.standard_normal((nq, d))).astype(dtype)
    return gal, qs


@pytest.mark.parametrize("mode_name", ["SIM_F16", "SIM_BF16", "SIM_BF16X3"])
def test_topk_batch_matches_oracle(torch_cuda, mode_name):
    """1,024 captions x 20,000 videos: every row resolved by the fused path, ids exact."""
    from cmve import engine, _lib
    gal, qs = _batch_case(41, 1024, 20000, 256)
    q = engine.RowSet(qs, with_lo=True)
    g = engine.RowSet(gal, with_lo=True)
    mode = getattr(_lib, mode_name)
    assert engine.topk_batch_plan(q, g, 10)[0]
    idx, sc, unres = engine.topk_batch(q, g, 10, mode)
    assert int(unres.item()) == 0
    _check(idx.cpu().numpy(), sc.cpu().numpy(), R.exact_scores64(qs, gal), 10)


def test_topk_batch_equals_dense(torch_cuda):
    """Fused and dense paths return identical ids and identical fp64 scores (f64 inputs, k = 25)."""
    from cmve import engine
    gal, qs = _batch_case(42, 700, 30000, 200, sigma=2.0, dtype=np.float64)
    q = engine.RowSet(qs, with_lo=True)
    g = engine.RowSet(gal, with_lo=True)
    a = engine.topk(q, g, 25, batch=True)
    b = engine.topk(q, g, 25, batch=False)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    _check(a[0], a[1], R.exact_scores64(qs, gal), 25)


def test_topk_batch_unresolved_rows_fall_back(torch_cuda):
    """Queries next to a 3,000-video near-duplicate cluster exceed the 512 kept entries (left
    unresolved, finished by cmve_topk); zero gallery rows (NaN columns) never enter a list."""
    from cmve import engine
    rng = np.random.default_rng(43)
    d, ng, nq = 256, 40000, 600
    base = rng.standard_normal(d)
    gal = rng.standard_normal((ng, d))
    gal[30000:33000] = base + 0.02 * rng.standard_normal((3000, d))  # outside the sample
    gal[::97] = 0.0
    qs = gal[rng.integers(0, ng, nq)] + 2.0 * rng.standard_normal((nq, d))
    qs[:40] = base + 0.5 * rng.standard_normal((40, d))
    q = engine.RowSet(qs, with_lo=True)
    g = engine.RowSet(gal, with_lo=True)
    _, _, unres = engine.topk_batch(q, g, 20)
    assert int(unres.item()) >= 40
    idx, sc = engine.topk(q, g, 20)
    _check(idx, sc, R.exact_scores64(qs, gal), 20)


def test_topk_batch_bench_shape(torch_cuda):
    """4,096 x 131,072 x 1024 (the bench shard, G256 persistent kernel): every row resolved;
    a sample of 48 rows checked against fp64."""
    import torch
    from cmve import engine
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(44)
    gal = torch.randn((131072, 1024), generator=gen, device=dev)
    pick = torch.randint(0, 131072, (4096,), generator=gen, device=dev)
    qs = gal[pick] + 10.0 * torch.randn((4096, 1024), generator=gen, device=dev)
    q = engine.RowSet(qs, eps=0.0, with_lo=True, device=dev)
    g = engine.RowSet(gal, eps=0.0, with_lo=True, device=dev)
    idx, sc, unres = engine.topk_batch(q, g, 10)
    assert int(unres.item()) == 0
    rows = np.arange(0, 4096, 4096 // 48)
    s = R.exact_scores64(qs[rows].cpu().numpy(), gal.cpu().numpy())
    _check(idx.cpu().numpy()[rows], sc.cpu().numpy()[rows], s, 10)


@pytest.mark.parametrize("nq,ng,d,k,qdt,gdt", [(517, 70001, 200, 1, np.float64, np.float32),
                                               (530, 140000, 96, 32, np.float32, np.float64),
                                               (1040, 9000, 1024, 17, np.float32, np.float32)])
def test_topk_batch_edge_shapes(torch_cuda, nq, ng, d, k, qdt, gdt):
    """Ragged query counts (not a multiple of the 16-query finish block), unpadded gallery sizes,
    k = 1 and k = 32 (the batch path's limit), mixed f32 / f64 raw rows: ids exact vs fp64."""
    from cmve import engine
    rng = np.random.default_rng(nq + k)
    gal = rng.standard_normal((ng, d)).astype(gdt)
    qs = (gal[rng.integers(0, ng, nq)] + 3.0 * rng.standard_normal((nq, d))).astype(qdt)
    q = engine.RowSet(qs, with_lo=True)
    g = engine.RowSet(gal, with_lo=True)
    ok, ns, _ = engine.topk_batch_plan(q, g, k)
    assert ok and ns <= ng // 4
    idx, sc = engine.topk(q, g, k)
    rows = np.arange(nq) if nq * ng <= 40_000_000 else np.linspace(0, nq - 1, 64).astype(int)
    s = R.exact_scores64(qs[rows], gal)
    _check(idx[rows], sc[rows], s, k)


def test_gallery_scorer_resident_buffers(torch_cuda):
    """GalleryScorer re-packs each new caption into its resident query buffers (per shape) and
    reuses its outputs: consecutive calls, 1- and 3-caption batches, all equal the oracle."""
    import torch
    from cmve.linas.inference import GalleryScorer
    rng = np.random.default_rng(12)
    gal = rng.standard_normal((6000, 192))
    sc = GalleryScorer(gal)
    for t in range(4):
        nq = 1 if t % 2 == 0 else 3
        caps = gal[rng.integers(0, 6000, nq)] + 0.9 * rng.standard_normal((nq, 192))
        arg = caps if t < 2 else torch.from_numpy(caps).cuda()
        idx = sc.topk_indices(arg, 7)
        expect = np.argsort(R.cal_error(gal, caps), axis=1, kind="stable")[:, :7]
        assert np.array_equal(idx, expect), f"call {t}"


@pytest.mark.parametrize("k,nc,ties", [(10, 5000, False), (64, 3000, True), (2048, 9000, True), (7, 5, True)])
def test_topk_dense_merge_kernel(torch_cuda, k, nc, ties):
    """K12f (cmve_topk_dense_merge) against numpy's stable sort of the same candidates by (score desc, id asc):
    a running best of k entries merged with a chunk of fp64 scores (ids j0 + c), exact ties (many rows share
    the k-th score), NaN (-> -inf, last) and -0.0 (== +0.0); the first chunk (kb = 0) and fewer candidates
    than k (ids -1 / -inf past them)."""
    import torch
    from cmve import engine
    from cmve._lib import lib, check
    rng = np.random.default_rng(k + nc)
    rows = 3
    s = rng.standard_normal((rows, nc))
    if ties:
        s = np.round(s, 1)  # ~60 distinct values: heavy ties at every rank
        s[:, ::17] = np.nan
        s[:, 5::23] = -0.0
        s[:, 6::23] = 0.0
    st = torch.from_numpy(s).cuda()

    def run(best_s, best_i, kb, chunk, j0):
        out_s = torch.empty((rows, k), dtype=torch.float64, device="cuda")
        out_i = torch.empty((rows, k), dtype=torch.int64, device="cuda")
        check(lib.cmve_topk_dense_merge(engine.handle(st.device), engine._ptr(best_s), engine._ptr(best_i), kb,
                                        engine._ptr(chunk), chunk.stride(0), rows, chunk.shape[1], j0, k,
                                        engine._ptr(out_s), engine._ptr(out_i)), "cmve_topk_dense_merge")
        return out_s.cpu().numpy(), out_i.cpu().numpy()

    def ref(vals, ids):
        v = np.where(np.isnan(vals), -np.inf, vals)
        o = np.lexsort((ids, -v))  # primary: score desc, then id asc
        return v[o][:k], ids[o][:k]

    # first chunk (no running best), then a second chunk merged with it
    h = nc // 2
    empty_s = torch.empty((rows, 1), dtype=torch.float64, device="cuda")
    empty_i = torch.empty((rows, 1), dtype=torch.int64, device="cuda")
    b_s, b_i = run(empty_s, empty_i, 0, st[:, :h].contiguous(), 0)
    kb = min(k, h)
    bs_t = torch.from_numpy(np.ascontiguousarray(b_s[:, :kb])).cuda()
    bi_t = torch.from_numpy(np.ascontiguousarray(b_i[:, :kb])).cuda()
    m_s, m_i = run(bs_t, bi_t, kb, st[:, h:].contiguous(), h)
    for r in range(rows):
        e_s, e_i = ref(s[r, :h], np.arange(h))
        n1 = len(e_i)
        assert np.array_equal(b_i[r, :n1], e_i) and np.array_equal(b_s[r, :n1], e_s)
        assert np.all(b_i[r, n1:] == -1)
        e_s, e_i = ref(s[r], np.arange(nc))
        n2 = len(e_i)
        assert np.array_equal(m_i[r, :n2], e_i) and np.array_equal(m_s[r, :n2], e_s)
