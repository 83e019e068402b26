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


def cirr_target_ranks(predicted_features: torch.Tensor, index_pooled: torch.Tensor, index_names: Sequence,
                      reference_names: Sequence, target_names: Sequence) -> np.ndarray:
    """1-based rank of each query's target after removing its reference video; 0 = never retrieved."""
    dev = predicted_features.device if torch.is_tensor(predicted_features) else engine.default_device()
    pos = {n: i for i, n in enumerate([int(v) for v in index_names])}
    tgt = [pos.get(int(t), -1) for t in target_names]
    ref = [pos.get(int(r), -1) for r in reference_names]
    q = engine.RowSet(predicted_features, eps=1e-12, with_lo=False, device=dev)
    g = engine.RowSet(index_pooled, eps=1e-12, with_lo=False, device=dev)
    row_gts = [[t] if t >= 0 else [] for t in tgt]
    ranks, _, _ = engine.gt_rank_counts(q, g, row_gts=row_gts)
    # the reference video is removed from the ranked list: drop it from the count when it outranks the target
    ref_gts = [[r] if r >= 0 else [] for r in ref]
    off_t, idx_t = engine.csr(row_gts, dev)
    off_r, idx_r = engine.csr(ref_gts, dev)
    s_t, _, _ = engine.gt_thresholds(q, g, off_t, idx_t, engine._lib.SIM_F16)
    s_r, _, _ = engine.gt_thresholds(q, g, off_r, idx_r, engine._lib.SIM_F16)
    s_t = s_t[:q.n].cpu().numpy()
    s_r = s_r[:q.n].cpu().numpy()
    out = ranks.astype(np.int64)
    for i in range(q.n):
        if tgt[i] < 0 or tgt[i] == ref[i]:
            out[i] = 0
        elif ref[i] >= 0 and s_r[i] > s_t[i]:
            out[i] -= 1
    return out


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
