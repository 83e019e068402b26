"""Golden vectors for the MultiFusion single-query scorer (MultiFusion/src/inference.py:26-66,124-136).

The reference's inference.py imports clip, decord and PIL (absent here), so it is NOT importable: the
glue of compute_cirr_val_metrics (normalize the index, reshape + F.adaptive_avg_pool2d of the middle
tokens, 1 - pred @ index.T, argsort, top-1 name) is restated below line by line with the reference's
own torch calls, and the combine runs on the REFERENCE's Combiner module (MultiFusion/src/combiner.py,
importable: torch only) with synth.combiner_state weights.  The CLIP text tower is replaced by a fixed
text feature (synth.multifusion_query), as the cmve test's stub clip_model returns.  Parity of the
glue is therefore pinned to this restatement only ("parity unpinned" against a reference run).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_multifusion_infer.py /root/reference
Writes tests/golden/multifusion_infer.npz (outputs only; inputs regenerate from the seed).
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

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
    for name, kw in (("c1280", {}), ("c640", {"channels": 640, "seed": 32})):
        high, mid, text, gallery, names = synth.multifusion_query(**kw)
        with torch.no_grad():
            # inference.py:133: index_features = concat(combiner.time_process(high_t.unsqueeze(0)))
            index_features = torch.cat([m.time_process(torch.from_numpy(g).unsqueeze(0)) for g in gallery])
            # inference.py:51-66
            index_features = F.normalize(index_features, dim=-1).float()
            ref_high = torch.from_numpy(high).unsqueeze(0)
            middle = torch.from_numpy(mid).float()
            middle = F.adaptive_avg_pool2d(middle.reshape(1, middle.shape[0], 18 * 18, -1),
                                           (16, index_features.shape[-1]))
            pred = m.combine_features((ref_high, middle), torch.from_numpy(text))
            scores = 1 - pred @ index_features.T
            order = torch.argsort(scores, dim=-1)
        out[f"{name}_pooled"] = middle.numpy()
        out[f"{name}_pred"] = pred.numpy()
        out[f"{name}_scores"] = scores.numpy()
        out[f"{name}_order"] = order.numpy()
        out[f"{name}_top1"] = np.array(names[int(order[0][0])])
    path = os.path.join(HERE, "multifusion_infer.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
