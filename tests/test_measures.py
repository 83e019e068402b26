"""Non-cosine measures row: cdist / jaccard errors of evaluation.py and the
order / euclidean / L1 / L2 / jaccard similarities of loss.py on the K10 all-pairs kernel.

Golden vectors: tests/golden/measures.npz, from the reference's own cal_error / cal_error_batch /
cal_simi and loss.py functions (tests/golden/make_golden_measures.py).
Tolerances: the scipy cdist branches are fp64 in the reference and fp64-accumulated here, so they
agree to ~1e-12 relative and their per-row orderings are identical; jaccard and the loss.py sims
are fp32 torch in the reference (fp32 sums over D), fp64-accumulated here and rounded once to
fp32, so they agree to 2e-5 relative (a few fp32 ulps of the reference's summation error).
"""
import numpy as np
import pytest
import torch

from oracle import measures as OM

EVAL = ["euclidean", "l1", "l2", "l1_norm", "l2_norm", "jaccard"]
SIMS = ["order_sim", "euclidean_sim", "L1_sim", "L1_sim_norm", "L2_sim", "L2_sim_norm", "jaccard_sim"]


def _eval_inputs(g, m):
    return (g["cap_p"], g["vid_p"]) if m == "jaccard" else (g["cap"], g["vid"])


def _sim_inputs(g, name):
    return (g["im_p"], g["s_p"]) if name == "jaccard_sim" else (g["im"], g["s"])


def _tol(m):
    return dict(rtol=2e-5, atol=1e-6) if "jaccard" in m or m in SIMS else dict(rtol=1e-12, atol=1e-12)


def test_oracle_matches_reference_golden(golden):
    g = golden("measures")
    for m in EVAL:
        c, v = _eval_inputs(g, m)
        np.testing.assert_allclose(OM.cal_error(v, c, m), g[f"cal_error_{m}"], **_tol(m), err_msg=m)
    np.testing.assert_allclose(OM.cal_error(g["vid_p"], g["cap_p"], "jaccard"), g["cal_error_batch_jaccard"],
                               **_tol("jaccard"))
    np.testing.assert_allclose(OM.cal_simi(g["cap_p"], g["vid_p"], "jaccard"), g["cal_simi_jaccard"],
                               **_tol("jaccard"))
    for name in SIMS:
        im, s = _sim_inputs(g, name)
        np.testing.assert_allclose(OM.LOSS_SIMS[name](im, s), g[f"loss_{name}"], **_tol(name), err_msg=name)


@pytest.mark.gpu
def test_cal_error_measures_match_reference_golden(golden):
    from cmve.linas import evaluation as E
    g = golden("measures")
    for m in EVAL:
        c, v = _eval_inputs(g, m)
        got = E.cal_error(v, c, m)
        want = g[f"cal_error_{m}"]
        if m == "jaccard":
            assert isinstance(got, torch.Tensor) and got.dtype == torch.float32
            got = got.numpy()
        else:
            assert got.dtype == np.float64
            assert np.array_equal(np.argsort(got, axis=1, kind="stable"), np.argsort(want, axis=1, kind="stable"))
        assert got.shape == want.shape
        np.testing.assert_allclose(got, want, **_tol(m), err_msg=m)
    got = E.cal_error_batch(g["vid_p"], g["cap_p"], "jaccard", batch_size=16)
    assert isinstance(got, np.ndarray) and got.dtype == np.float32
    np.testing.assert_allclose(got, g["cal_error_batch_jaccard"], **_tol("jaccard"))
    got = E.cal_simi(g["cap_p"], g["vid_p"], "jaccard")
    np.testing.assert_allclose(got.numpy(), g["cal_simi_jaccard"], **_tol("jaccard"))


@pytest.mark.gpu
def test_loss_sims_match_reference_golden(golden):
    from cmve.linas import loss as L
    g = golden("measures")
    for name in SIMS:
        im, s = _sim_inputs(g, name)
        got = getattr(L, name)(torch.from_numpy(im).cuda(), torch.from_numpy(s).cuda())
        assert got.dtype == torch.float32 and got.shape == (im.shape[0], s.shape[0])
        np.testing.assert_allclose(got.cpu().numpy(), g[f"loss_{name}"], **_tol(name), err_msg=name)
    for name in ("cosine", "order", "euclidean", "jaccard"):
        assert L.get_sim(name) is L.NAME_TO_SIM[name]
    x = torch.from_numpy(g["im"]).cuda().requires_grad_()
    with pytest.raises(NotImplementedError, match="forward-only"):
        L.order_sim(x, torch.from_numpy(g["s"]).cuda())


@pytest.mark.gpu
@pytest.mark.parametrize("metric", ["sq_l2", "l2", "l1", "order", "jaccard"])
def test_pairwise_kernel_edges(metric):
    """Tile / K-slab edges (1, 63, 64, 65 rows; D = 1, 31, 33), f32/f64 mixes, strided rows and
    empty inputs, against the fp64 oracle."""
    from cmve import engine
    from cmve import _lib
    code = {"sq_l2": _lib.PW_SQ_L2, "l2": _lib.PW_L2, "l1": _lib.PW_L1, "order": _lib.PW_ORDER,
            "jaccard": _lib.PW_JACCARD}[metric]
    rng = np.random.default_rng(7)
    for na, nb, d in [(1, 1, 1), (63, 65, 31), (64, 130, 33), (200, 7, 515)]:
        a = rng.standard_normal((na, d + 3))[:, :d]
        b = rng.standard_normal((nb, d))
        if metric == "jaccard":
            a, b = np.abs(a), np.abs(b)
        want = getattr(OM, metric)(a, b) * 0.5 - 2.0
        ta = torch.from_numpy(np.ascontiguousarray(rng.standard_normal((na, d + 3)))).cuda()[:, :d]
        ta.copy_(torch.from_numpy(a))
        assert ta.stride(0) == d + 3  # lda > d
        tb = torch.from_numpy(b).cuda().float()
        got = engine.pairwise(ta, tb, code, 0.5, -2.0, torch.float64).cpu().numpy()
        want32 = getattr(OM, metric)(a, b.astype(np.float32).astype(np.float64)) * 0.5 - 2.0
        np.testing.assert_allclose(got, want32, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5)
    z = engine.pairwise(torch.zeros((0, 8), device="cuda"), torch.zeros((5, 8), device="cuda"), code)
    assert z.shape == (0, 5)
