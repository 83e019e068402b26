"""Generate the golden vectors by importing the REFERENCE's own functions (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py /root/reference

The reference is read-only and never travels to the GPU box: this script runs here and
commits small .npz fixtures (inputs are regenerated from seeds by tests/golden/synth.py
where they are large).  Reference functions used (file:line in the reference tree):
  LINAS-engine/evaluation.py:17-21        cal_error
  LINAS-engine/util/metrics.py:106-157    get_gt, eval_q2m   (per-query rank = meanr of a 1-row call)
  LINAS-engine/util/metrics.py:61-102     t2v_map, v2t_map
  LINAS-engine/validate.py:15-54          cal_perf
  LINAS-engine/inference.py:78-79         cal_error + np.argsort(errors[0])[:topK]
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import synth  # noqa: E402


def _import_reference(ref_root):
    linas = os.path.join(ref_root, "LINAS-engine")
    sys.path.insert(0, linas)
    import evaluation  # noqa
    import validate  # noqa
    from util import metrics  # noqa
    return evaluation, validate, metrics


def per_query_ranks(metrics, scores, gts):
    """The reference's own eval_q2m on one row at a time: meanr of a 1-row call == that row's rank."""
    n = scores.shape[0]
    return np.array([int(metrics.eval_q2m(scores[i:i + 1], [gts[i]])[4]) for i in range(n)], np.int32)


def retrieval_case(evaluation, validate, metrics, videos, captions, video_ids, caption_ids, sample_rows=4):
    errors = evaluation.cal_error(videos, captions, 'cosine')
    v2t_gt, t2v_gt = metrics.get_gt(video_ids, caption_ids)
    v2t, t2v = validate.cal_perf(errors, v2t_gt, t2v_gt)
    t2v_lists = [t2v_gt[i] for i in range(len(caption_ids))]
    t2v_ranks = per_query_ranks(metrics, errors, t2v_lists)
    v2t_ranks = per_query_ranks(metrics, errors.T, v2t_gt)
    return dict(errors_sample=errors[:sample_rows].copy(), errors_dtype=str(errors.dtype),
                v2t=np.array(v2t, np.float64), t2v=np.array(t2v, np.float64),
                t2v_ranks=t2v_ranks, v2t_ranks=v2t_ranks,
                t2v_gt_flat=np.array([t2v_gt[i][0] for i in range(len(caption_ids))], np.int32),
                v2t_gt_lens=np.array([len(l) for l in v2t_gt], np.int32))


def _defined(scores, lists):
    """A row's argsort rank is independent of numpy's (implementation-defined) order among NaN
    unless every GT is NaN and the row holds more than one NaN."""
    out = np.ones(scores.shape[0], bool)
    for i, g in enumerate(lists):
        if g and np.all(np.isnan(scores[i, g])) and np.count_nonzero(np.isnan(scores[i])) > 1:
            out[i] = False
    return out


def nan_cases(evaluation, validate, metrics):
    """Case a (fp32): video 7 is zero (its caption v7#0 ranks a lone NaN GT in every t2v row but the
    zero caption's); caption v3#1 is zero and shares video 3 with two finite captions (a GT list
    mixing NaN and finite); videos 30-39 have no caption (empty v2t lists).  Case b (fp64): caption
    v5#0 is zero and is video 5's only caption (a lone NaN GT in the v2t direction)."""
    out = {}
    rng = np.random.default_rng(11)
    for tag, dtype in (("a", np.float32), ("b", np.float64)):
        nv, d = 40, 64
        v = rng.standard_normal((nv, d)).astype(dtype)
        cid = []
        for i in range(30):
            for k in range(3 if i == 3 else (2 if i % 4 == 0 else 1)):
                cid.append(f"v{i}#{k}")
        owner = np.array([int(c[1:].split("#")[0]) for c in cid])
        c = (v[owner] + dtype(1.5) * rng.standard_normal((len(cid), d))).astype(dtype)
        if tag == "a":
            v[7] = 0.0
            c[cid.index("v3#1")] = 0.0
        else:
            c[cid.index("v5#0")] = 0.0
        vid = [f"v{i}" for i in range(nv)]
        with np.errstate(invalid="ignore", divide="ignore"):
            errors = evaluation.cal_error(v, c, 'cosine')
            v2t_gt, t2v_gt = metrics.get_gt(vid, cid)
            t2v_lists = [t2v_gt.get(i, []) for i in range(len(cid))]
            t2v_ranks = per_query_ranks(metrics, errors, t2v_lists)
            v2t_ranks = per_query_ranks(metrics, errors.T, v2t_gt)
        out[f"{tag}_videos"] = v
        out[f"{tag}_captions"] = c
        out[f"{tag}_owner"] = owner.astype(np.int32)
        out[f"{tag}_t2v_ranks"] = t2v_ranks
        out[f"{tag}_v2t_ranks"] = v2t_ranks
        out[f"{tag}_t2v_defined"] = _defined(errors, t2v_lists)
        out[f"{tag}_v2t_defined"] = _defined(errors.T, v2t_gt)
    return out


def main(ref_root):
    evaluation, validate, metrics = _import_reference(ref_root)
    out = {}

    # (i) C1: 1000 x 1000 x 1024, sigma 10, float64 pipeline buffers
    v, c, vid, cid = synth.c1_embeddings()
    out["c1"] = retrieval_case(evaluation, validate, metrics, v, c, vid, cid)

    # (i') multi-GT v2t: 200 videos x 20 captions, D 128
    v, c, vid, cid = synth.multi_caption_embeddings()
    out["multi"] = retrieval_case(evaluation, validate, metrics, v, c, vid, cid)

    # (i'') small float32 inputs + a zero video row (NaN column, sorts last) -- inputs stored
    rng = np.random.default_rng(7)
    vs = rng.standard_normal((80, 256), dtype=np.float32)
    cs = (vs[:64] + np.float32(2.0) * rng.standard_normal((64, 256), dtype=np.float32)).astype(np.float32)
    vs[70] = 0.0
    vid = [f"v{i}" for i in range(80)]
    cid = [f"v{i}#0" for i in range(64)]
    with np.errstate(invalid="ignore", divide="ignore"):
        case = retrieval_case(evaluation, validate, metrics, vs, cs, vid, cid, sample_rows=64)
    case.update(videos=vs, captions=cs)
    out["small_f32"] = case

    # (ii) inference.py top-K: 16 fp32 queries x 20k fp64 gallery
    g64, q32, pick = synth.gallery_queries()
    top = np.stack([np.argsort(evaluation.cal_error(g64, q32[i:i + 1], 'cosine')[0])[:10] for i in range(q32.shape[0])])
    out["infer"] = dict(top10=top.astype(np.int64), pick=pick.astype(np.int64))

    # (iii) NaN cases (zero-norm rows: LINAS l2norm has no epsilon, evaluation.py:10-14), ranked by the
    # reference's eval_q2m (np.argsort puts NaN after every finite score)
    out["nan"] = nan_cases(evaluation, validate, metrics)

    for name, d in out.items():
        path = os.path.join(HERE, f"retrieval_{name}.npz")
        np.savez_compressed(path, **{k: np.asarray(v) for k, v in d.items()})
        print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
