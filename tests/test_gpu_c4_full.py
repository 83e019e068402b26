"""C4 (BASELINE configs[3]) at its configured size: the MultiFusion composed-query path over all 30,364 CIRR-val
queries in file order (batches of 32, the last one of 28 rows partial: MultiFusion/src/validate.py:207-208) against
the 44,493-video gallery with reference removal (validate.py:71-105), Combiner(640, 2560, 5120) with seeded
weights and synthetic features (no CLIP / dataset offline).  Property checks at full size:
  * combine_batches equals the reference's per-batch loop of combine_features bit for bit over every query;
  * the fused target ranks equal the oracle's fp64 scoring (oracle/retrieval.py cirr_target_ranks) on 256
    sampled queries, most of which have their reference scoring above the target (the removal matters);
  * rank 0 exactly for the queries whose target is their reference (removed with it, never retrieved)."""
import numpy as np
import pytest

from oracle import retrieval as R

pytestmark = pytest.mark.gpu

NQ, NV = 30364, 44493


def test_c4_full_size_properties():
    import torch
    from cmve.multifusion.combiner import Combiner
    from cmve.multifusion import validate as V
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = Combiner(640, 2560, 5120).to(dev).eval()
    gen = torch.Generator(device=dev).manual_seed(3)
    index = torch.randn((NV, 8, 640), generator=gen, device=dev)
    text = torch.randn((NQ, 640), generator=gen, device=dev)
    mid = torch.randn((NQ, 8, 16, 640), generator=gen, device=dev)
    ref = torch.randint(0, NV, (NQ,), generator=gen, device=dev)
    tgt = (ref + torch.randint(1, NV, (NQ,), generator=gen, device=dev)) % NV
    tgt[::97] = ref[::97]
    high = index[ref]
    pooled = V.normalize(V.time_process(index))
    with torch.no_grad():
        loop = torch.cat([m.combine_features((high[i:i + 32], mid[i:i + 32]), text[i:i + 32])
                          for i in range(0, NQ, 32)])
        fused = torch.cat([m.combine_batches((high[i:i + 8192], mid[i:i + 8192]), text[i:i + 8192])
                           for i in range(0, NQ, 8192)])
    assert NQ % 32 == 28 and torch.equal(fused, loop)
    del loop
    pred = V.normalize(fused)
    ranks = V.cirr_target_ranks(pred, pooled, list(range(NV)), ref.tolist(), tgt.tolist())
    assert np.array_equal(ranks == 0, (tgt == ref).cpu().numpy())
    idx = np.linspace(0, NQ - 1, 256).round().astype(np.int64)
    p64 = pred[torch.from_numpy(idx).to(dev)].double().cpu().numpy()
    g64 = pooled.double().cpu().numpy()
    r_s, t_s = ref.cpu().numpy()[idx], tgt.cpu().numpy()[idx]
    want = R.cirr_target_ranks(p64, g64, np.arange(NV), list(r_s), list(t_s))
    assert np.array_equal(ranks[idx], want)
    s = p64 @ g64.T
    above = int(np.count_nonzero(s[np.arange(256), r_s] > s[np.arange(256), t_s]))
    assert above > 64, above  # the reference removal changes the sampled ranks (the prediction leans on it)
