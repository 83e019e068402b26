"""Drop-in mirror of ``LINAS-engine/util/metrics.py`` (retrieval metrics) on libcmve.so.

  get_gt(video_ids, caption_ids)          metrics.py:106-120  (host; bucketed, same output)
  eval_q2m(scores, q2m_gts)               metrics.py:124-157  -> (r1, r5, r10, medr, meanr)
  t2v_map(c2i, t2v_gts)                   metrics.py:61-79
  v2t_map(c2i, v2t_gts)                   metrics.py:83-102
The per-row argsort of the reference is replaced by rank counting on the GPU:
position of item k in np.argsort(row) == #{j : e_j < e_k} on tie-free rows.
``scores`` that are an ``ErrorMatrix`` from cmve.linas.evaluation.cal_error are ranked
by the fused exact path (fp64 decisions, no matrix re-read).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import engine
from .._lib import lib, check, CMVE_F32, CMVE_F64  # noqa: F401
from .evaluation import ErrorMatrix


def get_gt(video_ids, caption_ids):
    buckets = {}
    for i, cap_id in enumerate(caption_ids):
        buckets.setdefault(cap_id.split('#', 1)[0], []).append(i)
    v2t_gt = [list(buckets.get(vid_id, [])) for vid_id in video_ids]
    t2v_gt = {}
    for i, t_gts in enumerate(v2t_gt):
        for t_gt in t_gts:
            t2v_gt.setdefault(t_gt, [])
            t2v_gt[t_gt].append(i)
    return v2t_gt, t2v_gt


def _lists(gts, n):
    if isinstance(gts, dict):
        return [gts[i] for i in range(n)]  # KeyError on a missing caption, like metrics.py:142
    return [gts[i] for i in range(n)]


def metrics_from_ranks(gt_ranks):
    gt_ranks = np.asarray(gt_ranks)
    n_q = gt_ranks.shape[0]
    r1 = 100.0 * len(np.where(gt_ranks <= 1)[0]) / n_q
    r5 = 100.0 * len(np.where(gt_ranks <= 5)[0]) / n_q
    r10 = 100.0 * len(np.where(gt_ranks <= 10)[0]) / n_q
    medr = np.median(gt_ranks)
    meanr = gt_ranks.mean()
    return (r1, r5, r10, medr, meanr)


def _fused_sets(scores):
    meta = getattr(scores, '_cmve', None) if isinstance(scores, ErrorMatrix) else None
    return meta


def gt_ranks(scores, q2m_gts):
    """1-based best-GT rank per query (metrics.py:137-147)."""
    n_q, n_m = scores.shape
    lists = _lists(q2m_gts, n_q)
    meta = _fused_sets(scores)
    if meta is not None:
        caps, vids, sign = meta
        if sign < 0:  # errors = -cos: rank by cos descending
            r, _, _ = engine.gt_rank_counts(caps, vids, row_gts=lists)
            return r.astype(np.int32)
    return engine.rank_from_matrix(scores, lists).astype(np.int32)


def eval_q2m(scores, q2m_gts):
    return metrics_from_ranks(gt_ranks(scores, q2m_gts))


def gt_positions(errors, lists, transposed=False):
    """1-based positions of every GT item of every query in the ascending sort of its row
    (columns when transposed); returns a list of int arrays aligned with ``lists``."""
    device = engine.default_device()
    e = engine.to_device(errors, device)
    n_rows, n_cols = e.shape
    off, idx = engine.csr(lists, device)
    pos = torch.zeros(max(int(off[-1].item()), 1), dtype=torch.int32, device=device)
    check(lib.cmve_gt_positions_from_matrix(engine.handle(device), engine._ptr(e), engine._dtype_code(e), n_rows,
                                            n_cols, e.stride(0), 1 if transposed else 0, engine._ptr(off),
                                            engine._ptr(idx), engine._ptr(pos)), "cmve_gt_positions_from_matrix")
    p = pos.cpu().numpy().astype(np.int64) + 1
    offs = off.cpu().numpy()
    return [p[offs[i]:offs[i + 1]] for i in range(len(lists))]


def ap_from_positions(positions):
    """APScorer on a ranked list (LINAS-engine/basic/metric.py:31-46) from the positions of its
    relevant items: the m-th relevant item at position p_m contributes m / p_m."""
    p = np.sort(np.asarray(positions, np.float64))
    if p.size == 0:
        return 0.0
    return float(np.sum(np.arange(1, p.size + 1) / p) / p.size)


def t2v_map(c2i, t2v_gts):
    """metrics.py:61-79: AP of the FIRST GT video of each caption (= 1 / its position)."""
    n_q = c2i.shape[0]
    firsts = [[_lists(t2v_gts, n_q)[i][0]] for i in range(n_q)]
    meta = _fused_sets(c2i)
    if meta is not None and meta[2] < 0:
        caps, vids, _ = meta
        r, _, _ = engine.gt_rank_counts(caps, vids, row_gts=firsts)
        return float(np.mean(1.0 / r))
    pos = gt_positions(c2i, firsts)
    return float(np.mean([ap_from_positions(p) for p in pos]))


def v2t_map(c2i, v2t_gts):
    """metrics.py:83-102: AP over all GT captions of each video (columns of c2i)."""
    n_v = c2i.shape[1]
    lists = _lists(v2t_gts, n_v)
    meta = _fused_sets(c2i)
    if meta is not None and meta[2] < 0:
        caps, vids, _ = meta
        if all(len(l) <= 1 for l in lists):
            _, c, _ = engine.gt_rank_counts(caps, vids, col_gts=lists)
            return float(np.mean([1.0 / c[j] if lists[j] else 0.0 for j in range(n_v)]))
        pos = engine.gt_positions_fused(vids, caps, lists)
        return float(np.mean([ap_from_positions(p) for p in pos]))
    pos = gt_positions(c2i, lists, transposed=True)
    return float(np.mean([ap_from_positions(p) for p in pos]))
