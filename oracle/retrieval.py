"""CPU oracle for the retrieval hot path (score -> rank -> R@K / mAP / top-K).

TEST INFRASTRUCTURE ONLY.  This module is a plain-numpy restatement of the
reference's CPU scoring path.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker / the
timed CPU baseline -- never as the product path (the product path lives in
``cross-modal-video-engine_amd/cmve`` and fails loudly without ``libcmve.so``).

Parity pin: every function here is checked against golden vectors captured by
importing the reference's own functions in the build container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``; see
``tests/test_oracle_golden.py``).

Citations are ``path:line`` relative to the reference tree
(WWWindrunner/Cross-Modal-Video-Engine).
"""
from __future__ import annotations

import numpy as np


# ---------------------------------------------------------------------------
# normalisation + scoring
# ---------------------------------------------------------------------------

def l2norm(X):
    """Row L2 normalisation with NO epsilon, dtype preserving.

    Follows ``LINAS-engine/evaluation.py:10-14`` (``np.linalg.norm(axis=1)``;
    ``1.0 * X / norm``).  A zero row yields NaN, exactly like the reference.
    """
    X = np.asarray(X)
    norm = np.linalg.norm(X, axis=1, keepdims=True)
    with np.errstate(invalid="ignore", divide="ignore"):
        return 1.0 * X / norm


def cal_error(videos, captions, measure="cosine"):
    """``errors[N_c, N_v] = -cos(caption, video)``.

    Follows ``LINAS-engine/evaluation.py:17-21`` (cosine branch): both sides are
    normalised in their own dtype and the product is taken in the promoted
    dtype (float32 x float64 -> float64, as ``np.dot`` does).
    """
    if measure != "cosine":
        raise NotImplementedError("oracle restates the cosine measure only (evaluation.py:18-21)")
    c = l2norm(captions)
    v = l2norm(videos)
    return -1 * np.dot(c, v.T)


def cal_simi(captions, videos, measure="cosine"):
    """``+cos`` twin of cal_error -- ``LINAS-engine/evaluation.py:75-84``."""
    if measure != "cosine":
        raise NotImplementedError
    return np.dot(l2norm(captions), l2norm(videos).T)


# ---------------------------------------------------------------------------
# ground truth + metrics
# ---------------------------------------------------------------------------

def get_gt(video_ids, caption_ids):
    """GT maps from ids.  Same output as ``LINAS-engine/util/metrics.py:106-120``.

    The reference is an O(N_v * N_c) double loop; this restatement buckets the
    caption ids by their ``'#'`` prefix (identical lists, identical order).
    """
    buckets = {}
    for i, cap_id in enumerate(caption_ids):
        buckets.setdefault(cap_id.split("#", 1)[0], []).append(i)
    v2t_gt = [list(buckets.get(vid_id, [])) for vid_id in video_ids]
    t2v_gt = {}
    for i, t_gts in enumerate(v2t_gt):
        for t_gt in t_gts:
            t2v_gt.setdefault(t_gt, [])
            t2v_gt[t_gt].append(i)
    return v2t_gt, t2v_gt


def gt_ranks(scores, q2m_gts):
    """Best (1-based) rank of any GT in ``np.argsort(scores[i])``.

    Follows the loop body of ``LINAS-engine/util/metrics.py:137-147``: rank starts
    at ``n_m + 1`` and takes the minimum over the GT list.
    """
    n_q, n_m = scores.shape
    ranks = np.zeros((n_q,), np.int32)
    for i in range(n_q):
        order = np.argsort(scores[i])
        rank = n_m + 1
        for k in q2m_gts[i]:
            rank = min(rank, int(np.where(order == k)[0][0]) + 1)
        ranks[i] = rank
    return ranks


def metrics_from_ranks(ranks):
    """``(r1, r5, r10, medr, meanr)`` from int ranks -- ``metrics.py:149-157``."""
    ranks = np.asarray(ranks)
    n_q = ranks.shape[0]
    r1 = 100.0 * len(np.where(ranks <= 1)[0]) / n_q
    r5 = 100.0 * len(np.where(ranks <= 5)[0]) / n_q
    r10 = 100.0 * len(np.where(ranks <= 10)[0]) / n_q
    medr = np.median(ranks)
    meanr = ranks.mean()
    return (r1, r5, r10, medr, meanr)


def eval_q2m(scores, q2m_gts):
    """``LINAS-engine/util/metrics.py:124-157``."""
    return metrics_from_ranks(gt_ranks(scores, q2m_gts))


def ap_score(sorted_labels):
    """``APScorer(0).score`` -- ``LINAS-engine/basic/metric.py:25-46`` (k=0 -> full length)."""
    nr_relevant = int(np.sum(np.asarray(sorted_labels) > 0))
    if nr_relevant == 0:
        return 0.0
    ap = 0.0
    rel = 0
    for i, lab in enumerate(sorted_labels):
        if lab >= 1:
            rel += 1
            ap += float(rel) / (i + 1.0)
    return ap / nr_relevant


def t2v_map(c2i, t2v_gts):
    """``LINAS-engine/util/metrics.py:61-79`` -- uses only the FIRST GT (:72)."""
    perf = []
    for i in range(c2i.shape[0]):
        labels = np.zeros(c2i.shape[1], np.int64)
        labels[t2v_gts[i][0]] = 1
        perf.append(ap_score(labels[np.argsort(c2i[i, :])]))
    return np.mean(perf)


def v2t_map(c2i, v2t_gts):
    """``LINAS-engine/util/metrics.py:83-102`` -- all GTs of a video."""
    perf = []
    for i in range(c2i.shape[1]):
        labels = np.zeros(c2i.shape[0], np.int64)
        for x in v2t_gts[i]:
            labels[x] = 1
        perf.append(ap_score(labels[np.argsort(c2i[:, i])]))
    return np.mean(perf)


def ap_from_positions(positions_1based):
    """AP of a ranked list given the 1-based positions of the relevant items.

    Equivalent to ``ap_score`` on the label vector (``basic/metric.py:31-46``):
    the m-th relevant item at position p_m contributes m / p_m.
    """
    p = np.sort(np.asarray(positions_1based, np.float64))
    if p.size == 0:
        return 0.0
    return float(np.sum(np.arange(1, p.size + 1) / p) / p.size)


def cal_perf(t2v_all_errors, v2t_gt, t2v_gt):
    """``LINAS-engine/validate.py:15-54`` minus logging / tensorboard."""
    (t2v_r1, t2v_r5, t2v_r10, t2v_medr, t2v_meanr) = eval_q2m(t2v_all_errors, t2v_gt)
    t2v_map_score = t2v_map(t2v_all_errors, t2v_gt)
    (v2t_r1, v2t_r5, v2t_r10, v2t_medr, v2t_meanr) = eval_q2m(t2v_all_errors.T, v2t_gt)
    v2t_map_score = v2t_map(t2v_all_errors, v2t_gt)
    return ((v2t_r1, v2t_r5, v2t_r10, v2t_medr, v2t_meanr, v2t_map_score),
            (t2v_r1, t2v_r5, t2v_r10, t2v_medr, t2v_meanr, t2v_map_score))


# ---------------------------------------------------------------------------
# inference.py scorer
# ---------------------------------------------------------------------------

def inference_topk(video_embs, cap_emb, topK=10):
    """Indices of the top-K videos for each caption row.

    ``LINAS-engine/inference.py:78-79``: ``errors = cal_error(video_embs, cap_emb)``
    then ``np.argsort(errors[0])[:topK]`` (applied here to every row).
    """
    errors = cal_error(video_embs, cap_emb)
    return np.stack([np.argsort(errors[i])[:topK] for i in range(errors.shape[0])])


def exact_scores64(q, g):
    """fp64 cosine of raw rows (normalise in fp64, then dot) -- the oracle's tie-free
    view of ``evaluation.py:18-21`` used for rank counting."""
    q = np.asarray(q, np.float64)
    g = np.asarray(g, np.float64)
    return l2norm(q) @ l2norm(g).T


def rank_counts(scores_hi_better, gts):
    """rank_i = 1 + #{j : s_ij > max_{k in GT(i), s_ik not NaN} s_ik}; no-GT rows: n_m + 1;
    rows whose every GT scores NaN: n_m.

    On tie-free rows this equals ``gt_ranks(-s, gts)`` (the argsort form of
    ``metrics.py:137-147``) wherever numpy's order is defined: ``np.argsort`` puts NaN after
    every finite score, so NaN never beats a GT and a lone NaN GT ranks last (n_m).  With
    several NaN in a row numpy's order among them is implementation-defined (its SIMD sort
    does not keep index order); the GT is then taken as the last.  This is the form the GPU
    path implements.
    """
    s = np.asarray(scores_hi_better)
    n_q, n_m = s.shape
    out = np.empty(n_q, np.int32)
    for i in range(n_q):
        g = list(gts[i]) if (not isinstance(gts, dict) or i in gts) else []
        if len(g) == 0:
            out[i] = n_m + 1
            continue
        sg = s[i, g]
        sg = sg[~np.isnan(sg)]
        if sg.size == 0:
            out[i] = n_m
            continue
        out[i] = 1 + int(np.count_nonzero(s[i] > sg.max()))
    return out


def argsort_defined(scores_hi_better, gts):
    """Rows whose reference rank (np.argsort form) is defined independently of numpy's order
    among NaN: some GT scores a number, or the row holds at most one NaN."""
    s = np.asarray(scores_hi_better)
    out = np.ones(s.shape[0], bool)
    for i in range(s.shape[0]):
        g = list(gts[i]) if (not isinstance(gts, dict) or i in gts) else []
        if g and np.all(np.isnan(s[i, g])) and np.count_nonzero(np.isnan(s[i])) > 1:
            out[i] = False
    return out


# ---------------------------------------------------------------------------
# MultiFusion scoring surface
# ---------------------------------------------------------------------------

def cirr_recalls(predicted, index_pooled, index_names, reference_names, target_names,
                 batch=32, ks=(1, 5, 10, 50)):
    """Recall@K of ``MultiFusion/src/validate.py:44-138`` (restated in numpy fp32).

    Per batch of 32 queries: ``dist = 1 - pred @ index.T`` (fp32), argsort,
    drop the reference video (exactly one occurrence), labels of the top-50
    against the target name, recall = 100 * mean over queries.
    ``index_pooled`` must already be ``F.normalize(time_process(index))``.
    """
    predicted = np.asarray(predicted, np.float32)
    index_pooled = np.asarray(index_pooled, np.float32)
    names = np.asarray(index_names)
    labels = []
    n = predicted.shape[0]
    for b0 in range(0, n, batch):
        p = predicted[b0:b0 + batch]
        dist = (np.float32(1) - p @ index_pooled.T).astype(np.float32)
        order = np.argsort(dist, axis=-1, kind="stable")
        sorted_names = names[order]
        for r in range(p.shape[0]):
            row = sorted_names[r]
            row = row[row != reference_names[b0 + r]]
            labels.append(row[:max(ks)] == target_names[b0 + r])
    labels = np.stack(labels)
    return tuple(float(labels[:, :k].sum() / len(labels) * 100) for k in ks)


def cirr_target_ranks(predicted, index_pooled, index_names, reference_names, target_names):
    """Rank (1-based) of the target after reference removal, fp64 tie-free form:
    1 + #{j != ref : s_j > s_target}; 0 if target == reference (never found)."""
    s = np.asarray(predicted, np.float64) @ np.asarray(index_pooled, np.float64).T
    names = np.asarray(index_names)
    out = np.empty(s.shape[0], np.int64)
    for i in range(s.shape[0]):
        if reference_names[i] == target_names[i]:
            out[i] = 0
            continue
        t = int(np.where(names == target_names[i])[0][0])
        keep = names != reference_names[i]
        out[i] = 1 + int(np.count_nonzero((s[i] > s[i, t]) & keep))
    return out
