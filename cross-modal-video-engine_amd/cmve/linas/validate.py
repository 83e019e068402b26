"""Drop-in mirror of ``LINAS-engine/validate.py`` ``cal_perf`` (+ ``norm_score``) on libcmve.so.

``cal_perf(t2v_all_errors, v2t_gt, t2v_gt, tb_logger=None, model=None)`` returns the
reference's two 6-tuples (validate.py:15-54).  When ``t2v_all_errors`` comes from
``cmve.linas.evaluation.cal_error`` both directions are ranked in ONE fused GEMM pass
(t2v = row counts, v2t = column counts) with fp64-exact decisions.
"""
from __future__ import annotations

import logging

import numpy as np

from .. import engine
from . import metrics
from .evaluation import ErrorMatrix


def norm_score(t2v_all_errors):
    """validate.py:7-11 (host elementwise)."""
    s = -t2v_all_errors
    s = s - np.min(s)
    s = s / np.max(s)
    return -s


def _log(tag, r1, r5, r10, medr, meanr, m):
    logging.info(" * %s:" % tag)
    logging.info(" * r_1_5_10, medr, meanr: {}".format([round(r1, 1), round(r5, 1), round(r10, 1), round(medr, 1),
                                                         round(meanr, 1)]))
    logging.info(" * recall sum: {}".format(round(r1 + r5 + r10, 1)))
    logging.info(" * mAP: {}".format(round(m, 4)))
    logging.info(" * " + '-' * 10)


def cal_perf(t2v_all_errors, v2t_gt, t2v_gt, tb_logger=None, model=None):
    n_c, n_v = t2v_all_errors.shape
    t2v_lists = metrics._lists(t2v_gt, n_c)
    v2t_lists = metrics._lists(v2t_gt, n_v)
    meta = getattr(t2v_all_errors, '_cmve', None) if isinstance(t2v_all_errors, ErrorMatrix) else None
    if meta is not None and meta[2] < 0:
        caps, vids, _ = meta
        t2v_ranks, v2t_ranks, _ = engine.gt_rank_counts(caps, vids, row_gts=t2v_lists, col_gts=v2t_lists)
        if all(len(l) == 1 for l in t2v_lists):
            t2v_map_score = float(np.mean(1.0 / t2v_ranks))
        else:
            t2v_map_score = metrics.t2v_map(t2v_all_errors, t2v_gt)
        if all(len(l) <= 1 for l in v2t_lists):
            v2t_map_score = float(np.mean([1.0 / v2t_ranks[j] if v2t_lists[j] else 0.0 for j in range(n_v)]))
        else:
            v2t_map_score = metrics.v2t_map(t2v_all_errors, v2t_gt)
    else:
        t2v_ranks = engine.rank_from_matrix(t2v_all_errors, t2v_lists)
        v2t_ranks = engine.rank_from_matrix(t2v_all_errors, v2t_lists, transposed=True)
        t2v_map_score = metrics.t2v_map(t2v_all_errors, t2v_gt)
        v2t_map_score = metrics.v2t_map(t2v_all_errors, v2t_gt)

    (t2v_r1, t2v_r5, t2v_r10, t2v_medr, t2v_meanr) = metrics.metrics_from_ranks(t2v_ranks.astype(np.int32))
    (v2t_r1, v2t_r5, v2t_r10, v2t_medr, v2t_meanr) = metrics.metrics_from_ranks(v2t_ranks.astype(np.int32))
    _log("Text to Video", t2v_r1, t2v_r5, t2v_r10, t2v_medr, t2v_meanr, t2v_map_score)
    _log("Video to text", v2t_r1, v2t_r5, v2t_r10, v2t_medr, v2t_meanr, v2t_map_score)
    if tb_logger is not None:
        step = getattr(model, 'Eiters', 0)
        for k, v in (('v2t_r1', v2t_r1), ('v2t_r5', v2t_r5), ('v2t_r10', v2t_r10), ('v2t_medr', v2t_medr),
                     ('v2t_meanr', v2t_meanr), ('t2v_r1', t2v_r1), ('t2v_r5', t2v_r5), ('t2v_r10', t2v_r10),
                     ('t2v_medr', t2v_medr), ('t2v_meanr', t2v_meanr), ('v2t_map', v2t_map_score),
                     ('t2v_map', t2v_map_score)):
            tb_logger.log_value(k, v, step=step)
    return ((v2t_r1, v2t_r5, v2t_r10, v2t_medr, v2t_meanr, v2t_map_score),
            (t2v_r1, t2v_r5, t2v_r10, t2v_medr, t2v_meanr, t2v_map_score))


def cal_perf_embeddings(video_embs, cap_embs, video_ids, caption_ids):
    """tester.py:133-139 in one call: get_gt -> fused two-direction rank -> cal_perf tuples,
    without materialising the N_c x N_v error matrix on host."""
    v2t_gt, t2v_gt = metrics.get_gt(video_ids, caption_ids)
    caps = engine.RowSet(np.asarray(cap_embs), eps=0.0, with_lo=False)
    vids = engine.RowSet(np.asarray(video_embs), eps=0.0, with_lo=False)
    n_c, n_v = caps.n, vids.n
    t2v_lists = metrics._lists(t2v_gt, n_c)
    t2v_ranks, v2t_ranks, _ = engine.gt_rank_counts(caps, vids, row_gts=t2v_lists, col_gts=v2t_gt)
    t2v = metrics.metrics_from_ranks(t2v_ranks)
    v2t = metrics.metrics_from_ranks(v2t_ranks)
    firsts = [[l[0]] for l in t2v_lists]
    if all(len(l) == 1 for l in t2v_lists):
        t2v_map = float(np.mean(1.0 / t2v_ranks))
    else:
        r, _, _ = engine.gt_rank_counts(caps, vids, row_gts=firsts)
        t2v_map = float(np.mean(1.0 / r))
    if all(len(l) <= 1 for l in v2t_gt):
        v2t_map = float(np.mean([1.0 / v2t_ranks[j] if v2t_gt[j] else 0.0 for j in range(n_v)]))
    else:
        pos = engine.gt_positions_fused(vids, caps, v2t_gt)
        v2t_map = float(np.mean([metrics.ap_from_positions(p) for p in pos]))
    return v2t + (v2t_map,), t2v + (t2v_map,)
