"""MultiFusion scoring surface (MultiFusion/src/validate.py, utils.py) on libcmve.so.

  time_process(fea)                       combiner.py:140-143      mean over frames (K2)
  element_wise_sum(image_features, text)  utils.py:61-69           normalize(image_features[0]) -- ignores text
  cirr_recalls(pred, index_features, index_names, reference_names, target_names)
                                          validate.py:44-138       -> (g1, g2, g3, r1, r5, r10, r50), g* = -1
  compute_cirr_val_metrics(...)           validate.py:27-143       same signature; predictions via
                                          generate_cirr_val_predictions (validate.py:167-272)
The reference sorts 32 x 44,493 distances per batch on the host (validate.py:71-105) and
drops the reference video before reading the top-50 labels.  Here the target's rank is
counted on the GPU with exact fp64 decisions:
    rank = 1 + #{ j != ref : s_j > s_target }      (target == reference -> never retrieved)
and recall@K = 100 * mean(rank <= K).
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch

from .. import engine
from ..linas.model import temporal_pool


def time_process(fea: torch.Tensor) -> torch.Tensor:
    """fea [N, F, D] -> mean over F (combiner.py:140-143)."""
    return temporal_pool(fea.to(torch.float32), "mean")


def normalize(x: torch.Tensor) -> torch.Tensor:
    """F.normalize(x, dim=-1) (eps 1e-12) on the GPU, fp32 out."""
    rs = engine.RowSet(x.detach().float(), eps=1e-12, with_lo=False, with_f16=False, device=x.device)
    return rs.normalized(torch.float32)


def element_wise_sum(image_features, text_features):
    """utils.py:61-69: returns normalize(image_features[0]) -- the text is ignored (reference quirk)."""
    return normalize(image_features[0])


def _as_int64(names) -> np.ndarray:
    """int(v) of every name (ints, numpy ints or numeric strings), vectorised when possible."""
    if isinstance(names, (list, tuple)):
        try:  # a list of Python ints: one pass, no intermediate object array
            return np.fromiter(names, np.int64, len(names))
        except (TypeError, ValueError, OverflowError):
            pass
    a = np.asarray(names)
    if a.dtype.kind in "iu":
        return a.astype(np.int64, copy=False).reshape(-1)
    try:
        return a.astype(np.int64).reshape(-1)
    except (TypeError, ValueError):
        return np.asarray([int(v) for v in names], np.int64)


class _NameIndex:
    """index_names -> row lookups, vectorised: the last row of a repeated name (as a {name: row}
    dict built in order), -1 when absent."""

    def __init__(self, index_names: Sequence):
        keys = _as_int64(index_names)
        self.lut = None
        if keys.size and keys.min() >= 0 and keys.max() < 4 * keys.size + 1024:
            # dense non-negative ids (the usual case): a direct table, the last row of a repeated id winning
            self.lut = np.full(int(keys.max()) + 1, -1, np.int64)
            np.maximum.at(self.lut, keys, np.arange(keys.size, dtype=np.int64))
            return
        self.order = np.argsort(keys, kind="stable")
        self.sorted = keys[self.order]

    def rows(self, names: Sequence) -> np.ndarray:
        want = _as_int64(names)
        if self.lut is not None:
            ok = (want >= 0) & (want < self.lut.size)
            return np.where(ok, self.lut[np.where(ok, want, 0)], -1)
        if self.sorted.size == 0:
            return np.full(want.shape, -1, np.int64)
        at = np.searchsorted(self.sorted, want, side="right") - 1
        atc = np.clip(at, 0, None)
        hit = (at >= 0) & (self.sorted[atc] == want)
        return np.where(hit, self.order[atc], -1)


def _positions(index_names: Sequence, names: Sequence) -> np.ndarray:
    """Row of each name in index_names (see _NameIndex)."""
    return _NameIndex(index_names).rows(names)


_WS = {}  # undecided-pair lists kept per device across validation passes (grown once, then reused)


def cirr_target_ranks(predicted_features: torch.Tensor, index_pooled: torch.Tensor, index_names: Sequence,
                      reference_names: Sequence, target_names: Sequence) -> np.ndarray:
    """1-based rank of each query's target after removing its reference video; 0 = never retrieved.
    One fused rank-count pass (exact fp64 decisions) plus the reference's own score:
        rank = 1 + #{j : s_j > s_target} - [s_ref > s_target]     (validate.py:76-87)"""
    dev = predicted_features.device if torch.is_tensor(predicted_features) else engine.default_device()
    ix = _NameIndex(index_names)
    tgt = ix.rows(target_names)
    ref = ix.rows(reference_names)
    q = engine.RowSet(predicted_features, eps=1e-12, with_lo=False, device=dev)
    g = engine.RowSet(index_pooled, eps=1e-12, with_lo=False, device=dev)
    mode = engine._lib.SIM_F16

    def one_gt(pos):
        off = torch.from_numpy(np.concatenate([[0], np.cumsum(pos >= 0)]).astype(np.int64)).to(dev)
        idx = torch.from_numpy(np.ascontiguousarray(pos[pos >= 0], np.int32) if (pos >= 0).any()
                               else np.zeros(1, np.int32)).to(dev)
        return off, idx

    s_t, hi, lo = engine.gt_thresholds(q, g, *one_gt(tgt), mode)
    s_r, _, _ = engine.gt_thresholds(q, g, *one_gt(ref), mode)
    ws = _WS.get(str(dev))
    if ws is None or ws.cap < 64 * (q.n + g.n):
        ws = _WS[str(dev)] = engine.RankWorkspace(dev, cap=max(1 << 16, 64 * (q.n + g.n)))
    for _attempt in range(4):
        cnt, _ = engine.rank_count_launch(q, g, mode, row=(s_t, hi, lo), ws=ws)
        ncand = ws.ncand()
        if not ws.overflowed():
            break
        ws.grow(ncand)
    else:
        raise engine._lib.CmveError("cirr_target_ranks: candidate list kept overflowing")
    n = q.n
    t_dev = torch.from_numpy(tgt).to(dev)
    r_dev = torch.from_numpy(ref).to(dev)
    ranks = cnt[:n].to(torch.int64) + 1 - ((r_dev >= 0) & (s_r[:n] > s_t[:n])).to(torch.int64)
    ranks = torch.where((t_dev < 0) | (t_dev == r_dev), torch.zeros_like(ranks), ranks)
    return ranks.cpu().numpy()


def cirr_recalls(predicted_features, index_features, index_names, reference_names, target_names, combiner=None):
    """validate.py:44-138 given the predicted (normalised) features and the raw index features
    [N, F, D]: index = normalize(time_process(index)), then recall@{1,5,10,50} with reference removal."""
    dev = engine.default_device()
    idx = torch.as_tensor(index_features).to(dev).float()
    pooled = time_process(idx) if idx.dim() == 3 else idx
    pred = torch.as_tensor(predicted_features).to(dev).float()
    ranks = cirr_target_ranks(pred, pooled, index_names, reference_names, target_names)
    found = ranks > 0
    rec = [float(100.0 * np.count_nonzero(found & (ranks <= k)) / len(ranks)) for k in (1, 5, 10, 50)]
    return (-1, -1, -1, rec[0], rec[1], rec[2], rec[3])


def generate_cirr_val_predictions(clip_model, relative_val_dataset, combining_function, index_names: List,
                                  index_features: torch.Tensor, tokenize=None, batch_size: int = 32):
    """validate.py:167-272: batches of 32 in dataset order (the Combiner's raw reshapes mix a batch,
    so the batching is part of the result); returns (predicted_features, reference_names, target_names)."""
    if tokenize is None:
        import clip  # OpenAI CLIP tokenizer; not installed in the build image
        tokenize = clip.tokenize
    dev = index_features.device
    name_to_feat = dict(zip([int(n) for n in index_names], index_features))
    preds, refs, tgts = [], [], []
    items = [relative_val_dataset[i] for i in range(len(relative_val_dataset))]
    for b0 in range(0, len(items), batch_size):
        batch = items[b0:b0 + batch_size]
        ref_names = [int(x[0]) for x in batch]
        tgt_names = [int(x[1]) for x in batch]
        captions = [x[2] for x in batch]
        middle = torch.stack([torch.as_tensor(x[4]) for x in batch]).to(dev).float()
        with torch.no_grad():
            text = clip_model.encode_text(tokenize(captions).to(dev)).float()
            ref_high = torch.stack([name_to_feat[n] for n in ref_names])
            p = combining_function((ref_high, middle), text)
        preds.append(normalize(p))
        refs += ref_names
        tgts += tgt_names
    return torch.cat(preds), refs, tgts


def compute_cirr_val_metrics(relative_val_dataset, clip_model, index_features, index_names, combining_function,
                             combiner, tokenize=None):
    """validate.py:27-143 (same signature + optional tokenizer)."""
    pred, refs, tgts = generate_cirr_val_predictions(clip_model, relative_val_dataset, combining_function,
                                                     index_names, index_features, tokenize)
    return cirr_recalls(pred, index_features, index_names, refs, tgts, combiner)
