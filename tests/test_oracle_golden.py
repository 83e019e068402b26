"""Oracle (CPU restatement) pinned against golden vectors captured from the reference."""
import numpy as np
import pytest

import synth
from oracle import retrieval as R


def _case(golden, name):
    return golden(f"retrieval_{name}")


@pytest.mark.parametrize("name", ["c1", "multi"])
def test_cal_perf_and_ranks(golden, name):
    g = _case(golden, name)
    if name == "c1":
        v, c, vid, cid = synth.c1_embeddings()
    else:
        v, c, vid, cid = synth.multi_caption_embeddings()
    errors = R.cal_error(v, c)
    np.testing.assert_allclose(errors[:g["errors_sample"].shape[0]], g["errors_sample"], rtol=0, atol=1e-12)
    v2t_gt, t2v_gt = R.get_gt(vid, cid)
    t2v_lists = [t2v_gt[i] for i in range(len(cid))]
    assert np.array_equal(R.gt_ranks(errors, t2v_lists), g["t2v_ranks"])
    assert np.array_equal(R.gt_ranks(errors.T, v2t_gt), g["v2t_ranks"])
    # the rank-count form (what the GPU implements) equals the argsort form on these tie-free inputs
    s = -errors
    assert np.array_equal(R.rank_counts(s, t2v_lists), g["t2v_ranks"])
    assert np.array_equal(R.rank_counts(s.T, v2t_gt), g["v2t_ranks"])
    v2t, t2v = R.cal_perf(errors, v2t_gt, t2v_gt)
    np.testing.assert_allclose(v2t, g["v2t"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(t2v, g["t2v"], rtol=0, atol=1e-12)


def test_small_f32_with_nan_column(golden):
    g = _case(golden, "small_f32")
    vs, cs = g["videos"], g["captions"]
    with np.errstate(invalid="ignore"):
        errors = R.cal_error(vs, cs)
    assert errors.dtype == np.float32 and str(g["errors_dtype"]) == "float32"
    np.testing.assert_array_equal(np.isnan(errors), np.isnan(g["errors_sample"]))
    np.testing.assert_allclose(errors, g["errors_sample"], rtol=0, atol=2e-6, equal_nan=True)
    v2t_gt, t2v_gt = R.get_gt([f"v{i}" for i in range(80)], [f"v{i}#0" for i in range(64)])
    v2t, t2v = R.cal_perf(errors, v2t_gt, t2v_gt)
    np.testing.assert_allclose(v2t, g["v2t"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(t2v, g["t2v"], rtol=0, atol=1e-9)


def test_inference_topk(golden):
    g = _case(golden, "infer")
    g64, q32, pick = synth.gallery_queries()
    assert np.array_equal(pick, g["pick"])
    top = R.inference_topk(g64, q32, 10)
    assert np.array_equal(top, g["top10"])


def test_ap_from_positions_matches_apscorer():
    rng = np.random.default_rng(0)
    for _ in range(50):
        n = int(rng.integers(1, 60))
        labels = (rng.random(n) < 0.2).astype(np.int64)
        pos = np.nonzero(labels)[0] + 1
        assert abs(R.ap_score(labels) - R.ap_from_positions(pos)) < 1e-12


def nan_case(g, tag):
    """Inputs and GT lists of retrieval_nan.npz case `tag` (ids v{i} / v{owner}#k, get_gt order)."""
    v, c, own = g[tag + "_videos"], g[tag + "_captions"], g[tag + "_owner"]
    t2v = [[int(o)] for o in own]
    v2t = [[i for i in range(c.shape[0]) if own[i] == j] for j in range(v.shape[0])]
    return v, c, t2v, v2t


@pytest.mark.parametrize("tag", ["a", "b"])
def test_nan_gt_ranks_match_reference(golden, tag):
    """Zero-norm rows (l2norm without eps -> NaN scores): the reference's eval_q2m ranks a lone NaN GT
    last (n_m) and takes the finite GT of a mixed list.  Where numpy's argsort order is defined (not
    several NaN in a row whose every GT is NaN), the oracle's count form == its argsort form == the
    reference; elsewhere the count form gives n_m (the GT taken as the last NaN)."""
    g = golden("retrieval_nan")
    v, c, t2v, v2t = nan_case(g, tag)
    with np.errstate(invalid="ignore", divide="ignore"):
        s = -R.cal_error(v, c)
    for scores, lists, key in ((s, t2v, "t2v"), (s.T, v2t, "v2t")):
        ref = g[f"{tag}_{key}_ranks"]
        ok = g[f"{tag}_{key}_defined"]
        assert np.array_equal(ok, R.argsort_defined(scores, lists))
        counts = R.rank_counts(scores, lists)
        assert np.array_equal(counts[ok], ref[ok])
        assert np.array_equal(R.gt_ranks(-scores, lists)[ok], ref[ok])
        assert np.all(counts[~ok] == scores.shape[1])
    # the fixture holds each case it was built for: a lone NaN GT ranked last, a mixed list, empty lists
    n_m = v.shape[0]
    assert any(np.isnan(s[i, l]).all() and g[f"{tag}_t2v_ranks"][i] == n_m for i, l in enumerate(t2v)) or tag == "b"
    assert tag == "a" or any(np.isnan(s[l, j]).all() and g["b_v2t_ranks"][j] == c.shape[0] for j, l in enumerate(v2t) if l)
