"""Drop-in mirror of ``LINAS-engine/evaluation.py`` backed by libcmve.so.

Same names, argument meaning and return types as the reference:
  l2norm(X)                                  evaluation.py:10-14
  cal_error(videos, captions, measure)       evaluation.py:17-36  -> ndarray[N_c, N_v] (= -cos; the
                                             euclidean / l1 / l2 / l1_norm / l2_norm / jaccard branches
                                             on the K10 all-pairs kernel)
  cal_error_batch(..., batch_size)           evaluation.py:41-72
  cal_simi(captions, videos, measure)        evaluation.py:75-84  -> ndarray[N_c, N_v] (= +cos)
  encode_vid / encode_text                   evaluation.py:88-171
The cosine matrix is computed on the GPU by the split-bf16 MFMA kernel (|err| ~1e-6,
within the north-star's 1e-4).  The returned array is an ``ErrorMatrix``: a plain
ndarray that also remembers the device-resident packed embeddings, so that
``cmve.linas.validate.cal_perf`` / ``cmve.linas.metrics.eval_q2m`` rank it with the
fused exact path (fp64-exact ranks, matrix never re-read) instead of the matrix path.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import engine
from .._lib import SIM_BF16X3, PW_L1, PW_L2, PW_JACCARD


class ErrorMatrix(np.ndarray):
    """ndarray of errors that carries the packed (captions, videos) sets it was made from."""

    _cmve = None  # (captions RowSet, videos RowSet, sign) -- dropped by any view/transform

    def __array_finalize__(self, obj):
        self._cmve = None


def _as_error_matrix(arr: np.ndarray, caps, vids, sign):
    out = arr.view(ErrorMatrix)
    out._cmve = (caps, vids, sign)
    return out


def _result_dtype(a, b):
    dt = np.result_type(np.asarray(a).dtype, np.asarray(b).dtype)
    return torch.float64 if dt == np.float64 else torch.float32


def l2norm(X):
    """Row L2 normalisation on the GPU, no epsilon (zero row -> NaN), dtype preserved."""
    X = np.asarray(X)
    rs = engine.RowSet(X, eps=0.0, with_lo=False)
    dt = torch.float64 if X.dtype == np.float64 else torch.float32
    return rs.normalized(dt).cpu().numpy()


def _cosine(videos, captions, sign):
    caps = engine.RowSet(np.asarray(captions), eps=0.0, with_lo=True)
    vids = engine.RowSet(np.asarray(videos), eps=0.0, with_lo=True)
    out = engine.sim_store(caps, vids, alpha=float(sign), beta=0.0, mode=SIM_BF16X3,
                           out_dtype=_result_dtype(captions, videos))
    return _as_error_matrix(out.cpu().numpy(), caps, vids, sign)


# scipy cdist branches of evaluation.py:22-33 / 56-67: measure -> (metric, alpha(D), beta), fp64 out
_CDIST = {
    'euclidean': (PW_L2, lambda D: 1.0, 0.0),
    'l2': (PW_L2, lambda D: 1.0, 0.0),
    'l1': (PW_L1, lambda D: 1.0, 0.0),
    'l1_norm': (PW_L1, lambda D: -1.0 / D, -1.0),
    'l2_norm': (PW_L2, lambda D: -1.0 / D, -1.0),
}


def _measure(videos, captions, measure):
    dev = engine.default_device()
    if measure in _CDIST:  # cdist works in fp64 whatever the input dtype
        metric, alpha, beta = _CDIST[measure]
        c = engine.to_device(np.asarray(captions), dev, torch.float64)
        v = engine.to_device(np.asarray(videos), dev, torch.float64)
        return engine.pairwise(c, v, metric, alpha(v.shape[1]), beta, torch.float64).cpu().numpy()
    if measure == 'jaccard':  # torch.Tensor(...) -> fp32 inputs, -jaccard_sim, returned as a torch tensor
        c = engine.to_device(np.asarray(captions), dev, torch.float32)
        v = engine.to_device(np.asarray(videos), dev, torch.float32)
        return engine.pairwise(c, v, PW_JACCARD, -1.0, 0.0, torch.float32).cpu()
    raise ValueError(f"cmve.cal_error: unknown measure {measure!r}")


def cal_error(videos, captions, measure='cosine'):
    """errors[N_c, N_v] (evaluation.py:17-36): -cos, or the cdist / jaccard branches."""
    if measure == 'cosine':
        return _cosine(videos, captions, -1)
    return _measure(videos, captions, measure)


def cal_error_batch(videos, captions, measure='cosine', batch_size=2000):
    """evaluation.py:41-72 -- the caption batching only bounds the reference's jaccard memory;
    the all-pairs kernel never materialises the [N_c, N_v, D] broadcast, so one call covers it
    (the jaccard result is a float32 ndarray here, as np.append makes it in the reference)."""
    out = cal_error(videos, captions, measure)
    return out.numpy() if measure == 'jaccard' else out


def cal_simi(captions, videos, measure='cosine'):
    """+cos(caption_i, video_j) or +jaccard as a float32 torch tensor (evaluation.py:75-84)."""
    if measure == 'cosine':
        return _cosine(videos, captions, +1)
    if measure == 'jaccard':
        dev = engine.default_device()
        c = engine.to_device(np.asarray(captions), dev, torch.float32)
        v = engine.to_device(np.asarray(videos), dev, torch.float32)
        return engine.pairwise(c, v, PW_JACCARD, 1.0, 0.0, torch.float32).cpu()
    raise ValueError(f"cmve.cal_simi: measure {measure!r} has no branch in the reference (evaluation.py:75-84)")


def _encode(encoder_call, data_loader, return_ids):
    embeddings = None
    ids = [''] * len(data_loader.dataset)
    for batch in data_loader:
        *datas, idxs, data_ids = batch
        emb = encoder_call(*datas)
        if embeddings is None:
            embeddings = np.zeros((len(data_loader.dataset), emb.size(1)))  # float64, as evaluation.py:102
        embeddings[list(idxs)] = emb.detach().cpu().numpy()
        for j, idx in enumerate(idxs):
            ids[idx] = data_ids[j]
    return (embeddings, ids) if return_ids else embeddings


def encode_vid(encoder, data_loader, return_ids=True):
    """evaluation.py:88-116: loader yields (datas, idxs, ids); float64 host buffer."""
    return _encode(lambda datas: encoder(datas), data_loader, return_ids)


def encode_text(encoder, data_loader, style, return_ids=True):
    """evaluation.py:119-171: 'distill_from_best_model' -> (datas, idxs, ids);
    'GT' -> (datas, support_datas, idxs, ids)."""
    if style == 'distill_from_best_model':
        return _encode(lambda datas: encoder(datas), data_loader, return_ids)
    if style == 'GT':
        return _encode(lambda datas, support: encoder(datas, support), data_loader, return_ids)
    raise ValueError(f"encode_text: unknown style {style!r}")
