"""GPU parity of the pool / projection / loss rows (through the C ABI) against the reference's
golden vectors (tests/golden/model_*.npz) and the oracle.  Floating-point tolerances are stated
per test (fp32 reference; split-bf16 projection ~1e-6 relative)."""
import numpy as np
import pytest

from oracle import heads as H

pytestmark = pytest.mark.gpu


def _sd(g):
    return {k[3:]: g[k] for k in g.files if k.startswith("sd_")}


def test_collate_frame(golden):
    import torch
    from cmve.linas.data import collate_frame
    g = golden("model_collate")
    frames = [torch.from_numpy(f) for f in np.split(g["frames"], np.cumsum(g["T"])[:-1])]
    (v, o, lens, m), idxs, ids = collate_frame([(f, i, f"v{i}") for i, f in enumerate(frames)])
    assert list(lens) == list(g["lengths"]) and list(idxs) == list(range(len(frames)))
    np.testing.assert_array_equal(v.cpu().numpy(), g["videos"])
    np.testing.assert_array_equal(m.cpu().numpy(), g["mask"])
    np.testing.assert_allclose(o.cpu().numpy(), g["origin"], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("pool", ["max", "mean"])
def test_video_level_features(golden, pool):
    """Pools of Video_multilevel_encoding.forward (model.py:143-176) around the reference's frozen
    GRU / Conv2d weights: HIP pools + torch conv vs the reference's forward output."""
    import torch
    from cmve.linas.model import video_level_features
    g = golden(f"model_venc_{pool}")
    col = golden("model_collate")
    sd = _sd(g)
    convs = []
    for k in range(4):
        w = torch.from_numpy(sd[f"convs1.{k}.weight"]).cuda()
        conv = torch.nn.Conv2d(1, w.shape[0], (w.shape[2], w.shape[3]), padding=(w.shape[2] - 1, 0)).cuda()
        conv.weight.data.copy_(w)
        conv.bias.data.copy_(torch.from_numpy(sd[f"convs1.{k}.bias"]))
        convs.append(conv)
    x = torch.from_numpy(g["gru_init_out"]).cuda()
    mask = torch.from_numpy(col["mask"]).cuda()
    origin = torch.from_numpy(col["origin"]).cuda()
    with torch.no_grad():
        f = video_level_features(x, mask, list(col["lengths"]), origin, convs, gru_pool=pool)
    np.testing.assert_allclose(f.cpu().numpy(), g["features"], rtol=1e-5, atol=2e-6)


def test_pool_modes_vs_oracle():
    import torch
    from cmve.linas.model import temporal_pool
    rng = np.random.default_rng(0)
    x = rng.standard_normal((37, 25, 2051)).astype(np.float32)   # TSN-like: 25 segments, odd F
    lens = rng.integers(1, 26, 37)
    mask = (np.arange(25)[None, :] < lens[:, None]).astype(np.float32)
    xt = torch.from_numpy(x).cuda()
    np.testing.assert_allclose(temporal_pool(xt, "mean").cpu().numpy(), H.pool_mean(x), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(temporal_pool(xt, "mean_valid", lens).cpu().numpy(), H.pool_mean_valid(x, lens),
                               rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(temporal_pool(xt, "masked_max", lens).cpu().numpy(), H.pool_masked_max(x, mask))
    np.testing.assert_array_equal(temporal_pool(xt, "max").cpu().numpy(), H.pool_max(x))
    # strided view (MultiFusion index features [N, 8, 640] sliced)
    big = torch.from_numpy(rng.standard_normal((9, 8, 700)).astype(np.float32)).cuda()[:, :, :640]
    np.testing.assert_allclose(temporal_pool(big, "mean").cpu().numpy(), big.cpu().numpy().mean(1), rtol=1e-5,
                               atol=1e-6)


@pytest.mark.parametrize("name", ["map2", "map3"])
def test_latent_mapping_eval(golden, name):
    import torch
    from cmve.linas.model import Latent_mapping
    g = golden(f"model_latent_{name}")
    layers = [int(v) for v in g["layers"]]
    lm = Latent_mapping(layers, 0.2).cuda()
    lm.load_state_dict({k: torch.from_numpy(v) for k, v in _sd(g).items()})
    lm.eval()
    y = lm(torch.from_numpy(g["x"]).cuda())
    np.testing.assert_allclose(y.cpu().numpy(), g["y"], rtol=0, atol=1e-5)  # fp32 ref ~1e-6 + split-bf16 per layer


@pytest.mark.parametrize("name", ["mv_sum_all", "mv_sum_all_b8", "mv_mean_all", "sum_all", "mv_sum_t2v", "mv_sum_v2t",
                                  "mean_all"])
def test_triplet_loss(golden, name):
    import torch
    from cmve.linas.loss import TripletLoss
    g = golden(f"model_triplet_{name}")
    m, mv, mean, dr = g["cfg"]
    direction = {1: "v2t", 2: "t2v", 3: "all"}[int(dr)]
    s = torch.from_numpy(g["s"]).cuda().requires_grad_(True)
    im = torch.from_numpy(g["im"]).cuda().requires_grad_(True)
    crit = TripletLoss(margin=float(m), measure='cosine', max_violation=bool(mv),
                       cost_style='mean' if mean else 'sum', direction=direction)
    loss = crit(s, im)
    loss.backward()
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(s.grad.cpu().numpy(), g["ds"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(im.grad.cpu().numpy(), g["dim"], rtol=0, atol=1e-5)


@pytest.mark.parametrize("B", [64, 256])
def test_infonce(golden, B):
    import torch
    from cmve.multifusion.loss import InfoNCE
    g = golden(f"model_infonce_{B}")
    res = {}
    for d in ("row", "col", "both"):
        P = torch.from_numpy(g["P"]).cuda().requires_grad_(True)
        T = torch.from_numpy(g["T"]).cuda().requires_grad_(True)
        loss = InfoNCE(100.0, d)(P, T)
        loss.backward()
        res[d] = (loss.item(), P.grad.cpu().numpy(), T.grad.cpu().numpy())
    np.testing.assert_allclose(res["row"][0], g["row"], rtol=1e-5)
    np.testing.assert_allclose(res["col"][0], g["col"], rtol=1e-5)
    np.testing.assert_allclose(res["both"][0], 0.5 * (g["row"] + g["col"]), rtol=1e-5)
    np.testing.assert_allclose(res["row"][1], g["dP_row"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(res["row"][2], g["dT_row"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(res["col"][1], g["dP_col"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(res["col"][2], g["dT_col"], rtol=0, atol=2e-5)
