"""MultiFusion scoring surface: the single-query scorer of MultiFusion/src/inference.py
(adaptive-avg-pool 18*18 -> 16, b = 1 combine, top-1) and validate.py's compute_cirr_val_metrics driven
end to end through the combining_function protocol with a stub CLIP text tower.

Parity: MultiFusion/src/{inference,validate}.py import clip / decord / PIL and are NOT importable here,
so their glue is pinned to a restatement (tests/golden/make_golden_multifusion_infer.py, which runs the
reference's own Combiner module for the combine) -- "parity unpinned" against a reference run.
Tolerances: pooling rtol 1e-6 (fp32 sums in another order), combined features atol 1e-5 (the
north-star's cosine bar), names / ranks exact.
"""
import numpy as np
import pytest

import synth
from oracle import combiner as OC
from oracle import retrieval as R

pytestmark = pytest.mark.gpu


class StubCLIP:
    """clip_model stand-in: encode_text maps a caption's token row to a fixed feature (the CLIP text
    tower is the frozen front end; the scorer only calls encode_text)."""

    def __init__(self, table):
        import torch
        self.table = torch.as_tensor(table).float().cuda()

    def encode_text(self, tokens):
        return self.table[tokens[:, 0].long()]


def _tokenize_by_index(captions):
    import torch
    return torch.tensor([[int(c.split("#")[1])] for c in captions])


@pytest.fixture(scope="module")
def combiner():
    import torch
    from cmve.multifusion.combiner import Combiner
    m = Combiner(640, 2560, 5120).cuda()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synth.combiner_state().items()})
    return m.eval()


@pytest.mark.parametrize("shape,out", [((3, 324, 1280), (16, 640)), ((8, 324, 640), (16, 640)),
                                       ((2, 324, 700), (16, 640)), ((4, 5, 9), (16, 7)), ((1, 17, 33), (1, 1))])
def test_adaptive_avg_pool2d_vs_torch(shape, out):
    import torch
    from cmve.multifusion.inference import adaptive_avg_pool2d
    x = torch.randn(*shape, generator=torch.Generator().manual_seed(sum(shape)))
    want = torch.nn.functional.adaptive_avg_pool2d(x[None], out)[0]
    got = adaptive_avg_pool2d(x.cuda(), out).cpu()
    torch.testing.assert_close(got, want, rtol=1e-6, atol=1e-6)
    # a strided (sliced) view takes the same path
    big = torch.randn(shape[0], shape[1], shape[2] + 5)
    got = adaptive_avg_pool2d(big.cuda()[:, :, :shape[2]], out).cpu()
    torch.testing.assert_close(got, torch.nn.functional.adaptive_avg_pool2d(big[None, :, :, :shape[2]], out)[0],
                               rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("name,kw", [("c1280", {}), ("c640", {"channels": 640, "seed": 32})])
def test_single_query_top1(golden, combiner, name, kw):
    import torch
    from cmve.multifusion import inference as MI
    g = golden("multifusion_infer")
    high, mid, text, gallery, names = synth.multifusion_query(**kw)
    middle = MI.adaptive_avg_pool2d(torch.from_numpy(mid).cuda().reshape(1, mid.shape[0], 324, -1), (16, 640))
    np.testing.assert_allclose(middle.cpu().numpy(), g[f"{name}_pooled"], rtol=1e-6, atol=1e-6)
    pred = combiner.combine_features((torch.from_numpy(high).cuda()[None], middle), torch.from_numpy(text).cuda())
    np.testing.assert_allclose(pred.cpu().numpy(), g[f"{name}_pred"], rtol=0, atol=1e-5)
    clip = StubCLIP(text)
    # clip.tokenize(str) -> [1, 77] (the reference passes the single modification text)
    tok = lambda caps: torch.zeros((1 if isinstance(caps, str) else len(caps), 1), dtype=torch.long)  # noqa: E731
    top1 = MI.retrieve_top1((torch.from_numpy(high), torch.from_numpy(mid)), "a modification", clip,
                            [torch.from_numpy(t) for t in gallery], names, combiner.combine_features, combiner,
                            tokenize=tok)
    assert top1 == str(g[f"{name}_top1"])
    # the same through compute_cirr_val_metrics with a precomputed (un-normalised) index
    index = combiner.time_process(torch.from_numpy(gallery).cuda())
    assert MI.compute_cirr_val_metrics((high, mid), "a modification", clip, index, names, combiner.combine_features,
                                       combiner, tokenize=tok) == top1


def test_validate_compute_cirr_val_metrics_end_to_end(combiner):
    """validate.py:27-143 through combining_function: batches of 32 (a partial last batch), a stub
    CLIP, the GPU ranks vs the CPU oracle's ranks on the oracle Combiner's predictions."""
    import torch
    from cmve.multifusion.validate import compute_cirr_val_metrics, normalize
    rng = np.random.default_rng(7)
    n_idx, n_q, f, d = 300, 70, 8, 640
    index_names = rng.permutation(5000)[:n_idx]
    index = rng.standard_normal((n_idx, f, d), dtype=np.float32)
    text_table = rng.standard_normal((n_q, d), dtype=np.float32)
    mids = rng.standard_normal((n_q, f, 16, d), dtype=np.float32)
    refs = rng.integers(0, n_idx, n_q)
    tgts = rng.integers(0, n_idx, n_q)
    tgts[3] = refs[3]   # target == reference: removed with the reference, never retrieved
    dataset = [(int(index_names[r]), int(index_names[t]), f"cap#{i}", [], mids[i])
               for i, (r, t) in enumerate(zip(refs, tgts))]
    index_t = torch.from_numpy(index).cuda()
    out = compute_cirr_val_metrics(dataset, StubCLIP(text_table), index_t, list(index_names),
                                   combiner.combine_features, combiner, tokenize=_tokenize_by_index)
    assert out[:3] == (-1, -1, -1)
    # oracle: fp64 Combiner per batch of 32 on the same inputs, then the CPU rank restatement
    sd = synth.combiner_state()
    preds = []
    for b0 in range(0, n_q, 32):
        sl = slice(b0, min(n_q, b0 + 32))
        preds.append(OC.combine_features(sd, index[refs[sl]], mids[sl], text_table[sl]))
    pred = np.concatenate(preds)
    pooled = index.astype(np.float64).mean(1)
    pooled /= np.maximum(np.linalg.norm(pooled, axis=1, keepdims=True), 1e-12)
    want = R.cirr_recalls(pred, pooled, index_names, index_names[refs], index_names[tgts])
    np.testing.assert_allclose(out[3:], want, rtol=0, atol=1e-9)
    assert normalize(torch.zeros(1, 4, device="cuda")).abs().sum().item() == 0  # F.normalize eps: no NaN
