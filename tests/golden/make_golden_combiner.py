"""(viii) Combiner golden vectors from the REFERENCE module (MultiFusion/src/combiner.py:81-180, importable:
it needs only torch), with deterministic weights from tests/golden/synth.py (no checkpoint stored).
b = 32 (validate.py:207-208 batch), b = 7 (a last partial batch) and b = 1 (inference.py:55);
combine_features outputs + forward logits for b = 32.
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_combiner.py /root/reference
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import synth  # noqa: E402


def main(ref_root):
    sys.path.insert(0, os.path.join(ref_root, "MultiFusion", "src"))
    import combiner as C  # noqa
    m = C.Combiner(640, 2560, 5120)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synth.combiner_state().items()})
    m.eval()
    out = {}
    with torch.no_grad():
        for b, seed in ((32, 21), (7, 22), (1, 23)):
            high, mid, text, tgt = synth.combiner_inputs(b, seed)
            pred = m.combine_features((torch.from_numpy(high), torch.from_numpy(mid)), torch.from_numpy(text))
            out[f"pred_b{b}"] = pred.numpy()
            if b == 32:
                logits = m((torch.from_numpy(high), torch.from_numpy(mid)), torch.from_numpy(text),
                           (torch.from_numpy(tgt),))
                out["logits_b32"] = logits.numpy()
        # batch-composition dependence: the first 7 queries of the b=32 batch run alone
        high, mid, text, _ = synth.combiner_inputs(32, 21)
        out["pred_b32_first7_alone"] = m.combine_features((torch.from_numpy(high[:7]), torch.from_numpy(mid[:7])),
                                                          torch.from_numpy(text[:7])).numpy()
    path = os.path.join(HERE, "combiner.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
