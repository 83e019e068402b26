"""MultiFusion ranking: recall@{1,5,10,50} with reference removal on the shipped val
split structure (first 256 triplets, 2,048-video sub-gallery, synthetic features)."""
import numpy as np
import pytest

import synth
from oracle import retrieval as R


def _case(golden):
    """Rebuild the inputs from the fixture's triplets (synth regenerates the features from the seed)."""
    g = golden("multifusion_rank")
    rows = [[str(i), str(r), str(t)] for i, r, t in zip(g["triplet_idx"], g["refs"], g["tgts"])]
    names, feats, pred, refs, tgts = synth.multifusion_ranking_case(rows)
    assert np.array_equal(names, g["names"]) and list(tgts) == list(g["tgts"])
    return g, names, feats, pred, refs, tgts


def test_oracle_recalls(golden):
    g, names, feats, pred, refs, tgts = _case(golden)
    pooled = feats.mean(axis=1)
    pooled = pooled / np.maximum(np.linalg.norm(pooled, axis=1, keepdims=True), 1e-12)
    rec = R.cirr_recalls(pred, pooled, names, refs, tgts)
    np.testing.assert_allclose(rec, g["recalls"], rtol=0, atol=1e-9)
    ranks = R.cirr_target_ranks(pred, pooled, names, refs, tgts)
    rec2 = [100.0 * np.count_nonzero((ranks > 0) & (ranks <= k)) / len(ranks) for k in (1, 5, 10, 50)]
    np.testing.assert_allclose(rec2, g["recalls"], rtol=0, atol=1e-9)
    assert ranks[5] == 0  # target == reference: removed with the reference, never retrieved


@pytest.mark.gpu
def test_gpu_cirr_recalls(golden):
    from cmve.multifusion.validate import cirr_recalls, cirr_target_ranks, time_process, normalize
    import torch
    g, names, feats, pred, refs, tgts = _case(golden)
    out = cirr_recalls(pred, feats, names, refs, tgts)
    assert out[:3] == (-1, -1, -1)
    np.testing.assert_allclose(out[3:], g["recalls"], rtol=0, atol=1e-9)
    pooled = normalize(time_process(torch.from_numpy(feats).cuda())).cpu().numpy()
    ranks = cirr_target_ranks(torch.from_numpy(pred).cuda(), torch.from_numpy(pooled).cuda(), names, refs, tgts)
    assert np.array_equal(ranks, R.cirr_target_ranks(pred, pooled, names, refs, tgts))


@pytest.mark.gpu
def test_element_wise_sum_ignores_text():
    import torch
    from cmve.multifusion.validate import element_wise_sum
    x = torch.randn(5, 640, device="cuda")
    out = element_wise_sum((x,), torch.randn(5, 640, device="cuda"))
    np.testing.assert_allclose(out.cpu().numpy(), torch.nn.functional.normalize(x, dim=-1).cpu().numpy(),
                               rtol=0, atol=1e-6)


def test_positions_lookup_matches_dict():
    """CIRR name -> gallery row lookup (vectorised): the last row of a repeated name, as the
    reference's {name: i} dict; absent names -1; numeric strings parsed like int(v)."""
    from cmve.multifusion.validate import _positions
    index = [5, 3, 9, 3, 7]
    table = {n: i for i, n in enumerate(index)}
    want = [3, 9, 4, 5, 7, 100]
    assert list(_positions(index, want)) == [table.get(n, -1) for n in want]
    assert list(_positions([str(v) for v in index], [str(v) for v in want])) == [table.get(n, -1) for n in want]
    assert list(_positions([], [1, 2])) == [-1, -1]
