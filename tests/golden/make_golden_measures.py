"""Golden vectors for the non-cosine measures row, produced by running the
REFERENCE's own functions on small seeded inputs:

  LINAS-engine/evaluation.py:17-38   cal_error        euclidean / l1 / l2 / l1_norm / l2_norm / jaccard
  LINAS-engine/evaluation.py:41-72   cal_error_batch  jaccard (batch_size 16: several sub-batches)
  LINAS-engine/evaluation.py:74-84   cal_simi         jaccard
  LINAS-engine/loss.py:13-73         order / euclidean / L1 / L1_norm / L2 / L2_norm / jaccard sims

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_measures.py /root/reference
Writes tests/golden/measures.npz (inputs included; they are small).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

EVAL_MEASURES = ["euclidean", "l1", "l2", "l1_norm", "l2_norm", "jaccard"]
LOSS_SIMS = ["order_sim", "euclidean_sim", "L1_sim", "L1_sim_norm", "L2_sim", "L2_sim_norm", "jaccard_sim"]


def inputs():
    """Ragged sizes (not multiples of the kernel's 64 x 64 tile or 32-deep K slab).  Non-negative
    features for jaccard (post-ReLU embeddings; a signed union can vanish and the ratio is then
    ill-conditioned in the reference's fp32)."""
    rng = np.random.default_rng(41)
    cap = rng.standard_normal((37, 203))          # fp64, like the encode_* buffers
    vid = rng.standard_normal((70, 203))
    cap_p = np.abs(rng.standard_normal((45, 131)))
    vid_p = np.abs(rng.standard_normal((66, 131)))
    im = rng.standard_normal((29, 96)).astype(np.float32)   # loss.py: fp32 torch batches
    s = rng.standard_normal((41, 96)).astype(np.float32)
    im_p = np.abs(im)
    s_p = np.abs(s)
    return dict(cap=cap, vid=vid, cap_p=cap_p, vid_p=vid_p, im=im, s=s, im_p=im_p, s_p=s_p)


def main(ref_root):
    sys.path.insert(0, os.path.join(ref_root, "LINAS-engine"))
    import torch
    import evaluation  # noqa
    import loss  # noqa
    x = inputs()
    out = dict(x)
    for m in EVAL_MEASURES:
        c, v = (x["cap_p"], x["vid_p"]) if m == "jaccard" else (x["cap"], x["vid"])
        e = evaluation.cal_error(v, c, m)
        out[f"cal_error_{m}"] = np.asarray(e.numpy() if hasattr(e, "numpy") else e)
    out["cal_error_batch_jaccard"] = np.asarray(evaluation.cal_error_batch(x["vid_p"], x["cap_p"], "jaccard",
                                                                           batch_size=16))
    out["cal_simi_jaccard"] = evaluation.cal_simi(x["cap_p"], x["vid_p"], "jaccard").numpy()
    for name in LOSS_SIMS:
        im, s = (x["im_p"], x["s_p"]) if name == "jaccard_sim" else (x["im"], x["s"])
        out[f"loss_{name}"] = getattr(loss, name)(torch.from_numpy(im), torch.from_numpy(s)).numpy()
    np.savez_compressed(os.path.join(HERE, "measures.npz"), **out)
    print({k: (v.shape, v.dtype) for k, v in out.items()})


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
