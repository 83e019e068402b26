"""Oracle restatements of the pool / projection / loss rows pinned to the reference's golden vectors."""
import numpy as np
import pytest

from oracle import heads as H


def _sd(g):
    return {k[3:]: g[k] for k in g.files if k.startswith("sd_")}


def test_collate_frame(golden):
    g = golden("model_collate")
    frames = np.split(g["frames"], np.cumsum(g["T"])[:-1])
    v, o, lens, m = H.collate_frame(frames)
    assert list(lens) == list(g["lengths"])
    np.testing.assert_array_equal(v, g["videos"])
    np.testing.assert_array_equal(m, g["mask"])
    np.testing.assert_allclose(o, g["origin"], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("pool", ["max", "mean"])
def test_video_encoder_pools(golden, pool):
    """gru pools of Video_multilevel_encoding.forward (model.py:152-158) from the reference's own GRU output."""
    g = golden(f"model_venc_{pool}")
    col = golden("model_collate")
    x = g["gru_init_out"].astype(np.float64)
    lengths = list(col["lengths"])
    gru = H.pool_mean_valid(x, lengths) if pool == "mean" else H.pool_masked_max(x, col["mask"])
    np.testing.assert_allclose(gru, g["features"][:, :x.shape[2]], rtol=1e-5, atol=1e-6)
    # the org (mean over all frames) slice is collate's origin
    np.testing.assert_allclose(g["features"][:, -col["origin"].shape[1]:], col["origin"], rtol=0, atol=0)


@pytest.mark.parametrize("name", ["map2", "map3"])
def test_latent_mapping(golden, name):
    g = golden(f"model_latent_{name}")
    y = H.latent_mapping_eval(g["x"], _sd(g), list(g["layers"]))
    np.testing.assert_allclose(y, g["y"], rtol=0, atol=2e-6)


@pytest.mark.parametrize("name", ["mv_sum_all", "mv_sum_all_b8", "mv_mean_all", "sum_all", "mv_sum_t2v", "mv_sum_v2t",
                                  "mean_all"])
def test_triplet(golden, name):
    g = golden(f"model_triplet_{name}")
    m, mv, mean, dr = g["cfg"]
    loss, ds, dim = H.triplet_loss(g["s"], g["im"], m, bool(mv), bool(mean), int(dr))
    np.testing.assert_allclose(loss, g["loss"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ds, g["ds"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(dim, g["dim"], rtol=0, atol=1e-5)


@pytest.mark.parametrize("B", [64, 256])
def test_infonce(golden, B):
    g = golden(f"model_infonce_{B}")
    row, col, dPr, dTr, dPc, dTc = H.infonce(g["P"], g["T"])
    np.testing.assert_allclose([row, col], [g["row"], g["col"]], rtol=1e-5)
    for a, b in ((dPr, "dP_row"), (dTr, "dT_row"), (dPc, "dP_col"), (dTc, "dT_col")):
        np.testing.assert_allclose(a, g[b], rtol=0, atol=2e-5)


@pytest.mark.parametrize("shape", [(3, 25, 32, 8, 8), (2, 3, 16, 7, 7), (4, 5, 8, 1, 1)])
def test_tsn_feature_extraction_against_torch_ops(shape):
    """MCT recognizer2d.py:76-83 restated (oracle.heads.tsn_feature_extraction) == the torch ops the
    reference calls there (nn.AdaptiveAvgPool2d(1), reshape, mean(axis=1)) on the same maps, in fp64.
    (MCT needs mmcv, absent: this pins the restatement to the ops, not to a run of the module.)"""
    import torch
    B, S, C, H_, W = shape
    x = np.random.default_rng(sum(shape)).standard_normal((B * S, C, H_, W))
    xt = torch.from_numpy(x)
    ref = torch.nn.AdaptiveAvgPool2d(1)(xt).reshape((B, S, -1)).mean(axis=1).numpy()
    np.testing.assert_allclose(H.tsn_feature_extraction(x, B), ref, rtol=0, atol=1e-14)
