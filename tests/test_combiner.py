"""Combiner.combine_features / forward: oracle and GPU path vs the reference module's
outputs (tests/golden/combiner.npz), deterministic weights from synth.combiner_state()."""
import numpy as np
import pytest

import synth
from oracle import combiner as OC


@pytest.fixture(scope="module")
def state():
    return synth.combiner_state()


@pytest.mark.parametrize("b,seed", [(32, 21), (7, 22), (1, 23)])
def test_oracle_combine(golden, state, b, seed):
    g = golden("combiner")
    high, mid, text, _ = synth.combiner_inputs(b, seed)
    np.testing.assert_allclose(OC.combine_features(state, high, mid, text), g[f"pred_b{b}"], rtol=0, atol=2e-6)


def test_oracle_batch_mixing_and_logits(golden, state):
    g = golden("combiner")
    high, mid, text, tgt = synth.combiner_inputs(32, 21)
    alone = OC.combine_features(state, high[:7], mid[:7], text[:7])
    np.testing.assert_allclose(alone, g["pred_b32_first7_alone"], rtol=0, atol=2e-6)
    assert np.abs(alone - g["pred_b32"][:7]).max() > 1e-3  # the reference's batch dependence is real
    np.testing.assert_allclose(OC.forward_logits(state, high, mid, text, tgt), g["logits_b32"], rtol=0, atol=2e-4)


@pytest.mark.gpu
def test_gpu_combiner(golden, state):
    import torch
    from cmve.multifusion.combiner import Combiner
    g = golden("combiner")
    m = Combiner(640, 2560, 5120).cuda()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()})
    m.eval()
    for b, seed in ((32, 21), (7, 22), (1, 23)):
        high, mid, text, tgt = synth.combiner_inputs(b, seed)
        pred = m.combine_features((torch.from_numpy(high).cuda(), torch.from_numpy(mid).cuda()),
                                  torch.from_numpy(text).cuda())
        np.testing.assert_allclose(pred.cpu().numpy(), g[f"pred_b{b}"], rtol=0, atol=1e-5)
        if b == 32:
            logits = m((torch.from_numpy(high).cuda(), torch.from_numpy(mid).cuda()), torch.from_numpy(text).cuda(),
                       (torch.from_numpy(tgt).cuda(),))
            np.testing.assert_allclose(logits.cpu().numpy(), g["logits_b32"], rtol=0, atol=1e-3)
    high, mid, text, _ = synth.combiner_inputs(32, 21)
    alone = m.combine_features((torch.from_numpy(high[:7]).cuda(), torch.from_numpy(mid[:7]).cuda()),
                               torch.from_numpy(text[:7]).cuda())
    np.testing.assert_allclose(alone.cpu().numpy(), g["pred_b32_first7_alone"], rtol=0, atol=1e-5)


@pytest.mark.gpu
def test_gpu_combine_batches_equals_batch_loop(state):
    """combine_batches (all full 32-row batches in one pass, per-batch attention layout rebuilt) is
    bit-identical to validate.py's loop of combine_features over consecutive batches of 32, the
    last partial batch (7 rows) included; and it still mixes rows within each batch only."""
    import torch
    from cmve.multifusion.combiner import Combiner
    m = Combiner(640, 2560, 5120).cuda()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()})
    m.eval()
    parts = [synth.combiner_inputs(32, 31 + i)[:3] for i in range(3)] + [synth.combiner_inputs(7, 40)[:3]]
    high, mid, text = (torch.from_numpy(np.concatenate([p[j] for p in parts])).cuda() for j in range(3))
    loop = torch.cat([m.combine_features((high[i:i + 32], mid[i:i + 32]), text[i:i + 32])
                      for i in range(0, high.shape[0], 32)])
    fused = m.combine_batches((high, mid), text, batch_size=32)
    assert torch.equal(loop, fused)
