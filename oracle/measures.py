"""CPU oracle for the non-cosine measures.

TEST INFRASTRUCTURE ONLY.  A plain-numpy fp64 restatement of the reference's all-pairs distance
and similarity matrices.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it, and only as the checker / timed CPU baseline; the product path
(``cmve.linas.evaluation`` / ``cmve.linas.loss`` on the K10 kernel ``cmve_pairwise``) never does.

Parity pin: checked against ``tests/golden/measures.npz``, produced by the reference's own
``evaluation.cal_error`` / ``cal_error_batch`` / ``cal_simi`` and ``loss.py`` similarity functions
(``tests/golden/make_golden_measures.py``; ``tests/test_measures.py``).

Citations are ``path:line`` in the reference tree.
"""
from __future__ import annotations

import numpy as np


def _diff(a, b):
    """[na, nb, D] of b_j - a_i in fp64 (the YmX of LINAS-engine/loss.py:16-17)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return b[None, :, :] - a[:, None, :]


def sq_l2(a, b):
    return np.einsum("ijk,ijk->ij", d := _diff(a, b), d)


def l2(a, b):
    """scipy cdist 'euclidean' (evaluation.py:23,27)."""
    return np.sqrt(sq_l2(a, b))


def l1(a, b):
    """scipy cdist 'minkowski' p=1 (evaluation.py:25)."""
    return np.abs(_diff(a, b)).sum(-1)


def order(a, b):
    """sqrt(sum max(0, b - a)^2) (loss.py:16-18)."""
    return np.sqrt((np.maximum(_diff(a, b), 0.0) ** 2).sum(-1))


def jaccard(a, b):
    """sum min / sum max (loss.py:65-73)."""
    a = np.asarray(a, np.float64)[:, None, :]
    b = np.asarray(b, np.float64)[None, :, :]
    return np.minimum(a, b).sum(-1) / np.maximum(a, b).sum(-1)


def cal_error(videos, captions, measure):
    """LINAS-engine/evaluation.py:17-38, non-cosine branches: errors[caption, video]."""
    D = np.asarray(videos).shape[1]
    if measure in ("euclidean", "l2"):
        return l2(captions, videos)
    if measure == "l1":
        return l1(captions, videos)
    if measure == "l1_norm":
        return -l1(captions, videos) / D - 1
    if measure == "l2_norm":
        return -l2(captions, videos) / D - 1
    if measure == "jaccard":  # the reference computes this one in torch fp32
        return -jaccard(np.float32(captions), np.float32(videos))
    raise ValueError(measure)


def cal_simi(captions, videos, measure):
    """LINAS-engine/evaluation.py:74-84 (jaccard branch)."""
    assert measure == "jaccard"
    return jaccard(np.float32(captions), np.float32(videos))


# LINAS-engine/loss.py:13-73: score[i_im, j_s]
LOSS_SIMS = {
    "order_sim": lambda im, s: -order(im, s),
    "euclidean_sim": lambda im, s: -sq_l2(im, s),
    "L1_sim": lambda im, s: -l1(im, s),
    "L1_sim_norm": lambda im, s: l1(im, s) / np.shape(im)[1] - 1,
    "L2_sim": lambda im, s: -sq_l2(im, s),
    "L2_sim_norm": lambda im, s: sq_l2(im, s) / np.shape(im)[1] - 1,
    "jaccard_sim": lambda im, s: jaccard(im, s),
}
