"""Drop-in mirror of ``LINAS-engine/evaluation.py`` backed by libcmve.so.

Same names, argument meaning and return types as the reference:
  l2norm(X)                                  evaluation.py:10-14
  cal_error(videos, captions, measure)       evaluation.py:17-36  -> ndarray[N_c, N_v] (= -cos)
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
from .._lib import SIM_BF16X3


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


def cal_error(videos, captions, measure='cosine'):
    """errors[N_c, N_v] = -cos(caption_i, video_j)  (evaluation.py:17-21)."""
    if measure == 'cosine':
        return _cosine(videos, captions, -1)
    raise NotImplementedError(
        f"cmve.cal_error: measure {measure!r} is not on the MI355X hot path yet (cosine only; "
        "euclidean/l1/l2/jaccard are SURVEY section 8f 'next' item 4)")


def cal_error_batch(videos, captions, measure='cosine', batch_size=2000):
    """evaluation.py:41-72 -- the batching only matters for the jaccard branch."""
    return cal_error(videos, captions, measure)


def cal_simi(captions, videos, measure='cosine'):
    """+cos(caption_i, video_j)  (evaluation.py:75-84)."""
    if measure == 'cosine':
        return _cosine(videos, captions, +1)
    raise NotImplementedError(f"cmve.cal_simi: measure {measure!r} not supported (cosine only)")


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
