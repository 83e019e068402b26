"""cmve_rank_fixup_tiled: the undecided pairs regrouped by (gallery super-bucket, query tile) before the fp64
re-score.  The counts are integer increments, so every grouping must give the plain bucket walk's counts bit for
bit (the ranking of MultiFusion/src/validate.py:71-105 and LINAS-engine/util/metrics.py:137-147)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _crowded(seed, n_q, n_g, d, n_centers=24, noise=0.04):
    """Rows around a few centres: the scores crowd around the GT scores, so tens of thousands of pairs fall
    inside the fp16 band (the CIRR ranking's situation, at test size)."""
    rng = np.random.default_rng(seed)
    cen = rng.standard_normal((n_centers, d)).astype(np.float32)
    cq = rng.integers(0, n_centers, n_q)
    cg = rng.integers(0, n_centers, n_g)
    q = cen[cq] + noise * rng.standard_normal((n_q, d)).astype(np.float32)
    g = cen[cg] + noise * rng.standard_normal((n_g, d)).astype(np.float32)
    by_c = [np.flatnonzero(cg == c) for c in range(n_centers)]
    row_gts = [[int(rng.choice(by_c[c]))] if by_c[c].size else [] for c in cq]
    col_gts = [[] for _ in range(n_g)]
    for i, l in enumerate(row_gts):
        for j in l:
            col_gts[j].append(i)
    return q, g, row_gts, col_gts


def _counts(engine, _lib, q, g, row, col, tiled):
    ws = engine.RankWorkspace(q.device, cap=1 << 22)
    rc, cc = engine.rank_count_launch(q, g, _lib.SIM_F16, row=row, col=col, ws=ws, tiled=tiled)
    assert not ws.overflowed()
    cc = cc[:g.n].cpu().numpy().copy() if cc is not None else None
    return rc[:q.n].cpu().numpy().copy(), cc, ws.ncand()


@pytest.mark.parametrize("n_q,n_g", [(2600, 3000), (700, 1900)])
def test_tiled_fixup_equals_plain(n_q, n_g):
    from cmve import engine, _lib
    qx, gx, row_gts, col_gts = _crowded(11, n_q, n_g, 640)
    q = engine.RowSet(qx, with_lo=False)
    g = engine.RowSet(gx, with_lo=False)
    row = engine.gt_thresholds(q, g, *engine.csr(row_gts, q.device), _lib.SIM_F16)
    col = engine.gt_thresholds(g, q, *engine.csr(col_gts, q.device), _lib.SIM_F16)
    rc0, cc0, nc = _counts(engine, _lib, q, g, row, col, None)
    assert nc > 20000, nc  # the case must exercise the walk
    # group sizes: the library's choice, one bucket, a group that does not divide the bucket count, more than all
    for group in (0, 1, 3, 5, 64):
        rc, cc, nc1 = _counts(engine, _lib, q, g, row, col, group)
        assert nc1 == nc
        assert np.array_equal(rc, rc0), group
        assert np.array_equal(cc, cc0), group
    # one direction only (the CIRR ranking's form)
    rc, _, _ = _counts(engine, _lib, q, g, row, None, 0)
    assert np.array_equal(rc, rc0)


def test_tiled_fixup_against_fp64():
    """Ranks from the tiled walk against an independent fp64 scoring of every pair."""
    from cmve import engine, _lib
    qx, gx, row_gts, _ = _crowded(12, 900, 1300, 640)
    q = engine.RowSet(qx, with_lo=False)
    g = engine.RowSet(gx, with_lo=False)
    row = engine.gt_thresholds(q, g, *engine.csr(row_gts, q.device), _lib.SIM_F16)
    rc, _, _ = _counts(engine, _lib, q, g, row, None, 0)
    qn = qx.astype(np.float64)
    gn = gx.astype(np.float64)
    s = (qn @ gn.T) / np.linalg.norm(qn, axis=1)[:, None] / np.linalg.norm(gn, axis=1)[None, :]
    for i in range(0, 900, 7):
        t = s[i, row_gts[i][0]]
        assert rc[i] == int(np.count_nonzero(s[i] > t)), i


def test_tiled_fixup_scratch_checked():
    from cmve import engine, _lib
    qx, gx, row_gts, _ = _crowded(13, 300, 600, 64)
    q = engine.RowSet(qx, with_lo=False)
    g = engine.RowSet(gx, with_lo=False)
    sgt, hi, lo = engine.gt_thresholds(q, g, *engine.csr(row_gts, q.device), _lib.SIM_F16)
    ws = engine.RankWorkspace(q.device, cap=1 << 16)
    cnt = torch.empty(q.n_pad, dtype=torch.int32, device=q.device)
    C = engine.C
    h = engine.handle(q.device)
    engine.check(engine.lib.cmve_rank_mfma(h, C.byref(q.desc), C.byref(g.desc), _lib.SIM_F16, _lib.DIR_ROW,
                                           engine._ptr(hi), engine._ptr(lo), None, None, engine._ptr(cnt), None,
                                           engine._ptr(ws.cand), ws.cap, engine._ptr(ws.count)), "cmve_rank_mfma")
    need = int(engine.lib.cmve_rank_fixup_tiled_scratch(C.byref(q.desc), C.byref(g.desc), ws.cap, 0))
    assert need > ws.cap
    small = torch.empty(need - 1, dtype=torch.int64, device=q.device)
    with pytest.raises(_lib.CmveError, match="scratch holds"):
        engine.check(engine.lib.cmve_rank_fixup_tiled(h, C.byref(q.desc), C.byref(g.desc), _lib.DIR_ROW,
                                                      engine._ptr(sgt), None, engine._ptr(cnt), None,
                                                      engine._ptr(ws.cand), ws.cap, engine._ptr(ws.count),
                                                      engine._ptr(small), small.numel(), 0), "cmve_rank_fixup_tiled")
    with pytest.raises(_lib.CmveError, match="group"):
        engine.check(engine.lib.cmve_rank_fixup_tiled(h, C.byref(q.desc), C.byref(g.desc), _lib.DIR_ROW,
                                                      engine._ptr(sgt), None, engine._ptr(cnt), None,
                                                      engine._ptr(ws.cand), ws.cap, engine._ptr(ws.count),
                                                      engine._ptr(small), small.numel(), 65), "cmve_rank_fixup_tiled")
    torch.cuda.synchronize()
