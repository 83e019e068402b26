"""Single-query composed retrieval of MultiFusion/src/inference.py on libcmve.so.

  adaptive_avg_pool2d(x, (OH, OW))          F.adaptive_avg_pool2d (inference.py:58-59), K2 kernel
  compute_cirr_val_metrics(ref_vdo_feature, mod_text, clip_model, index_features, index_names,
                           combining_function, combiner)
                                            inference.py:26-66 -> the top-1 index name
  retrieve_top1(ref_vdo_feature, mod_text, clip_model, target_features, tar_list,
                combining_function, combiner)
                                            inference.py:124-149 (cirr_val_retrieval) from features:
                                            index = time_process(target high features), then the above

The reference's query is one reference video (high features [T, D], middle tokens [T, 18*18, C]
reshaped to [1, T, 324, C] and adaptive-average-pooled to [1, T, 16, D]) plus a modification text
encoded by CLIP; ``combining_function`` combines them (b = 1) and the gallery is ranked by
``1 - pred @ normalize(index).T`` with ``torch.argsort``; the first name is returned.  Here the
gallery is normalised and packed once into HBM and the top-1 comes from the exact top-k kernel
(fp64 re-score of the error band; ties -> the lower index).  Decoding the videos and the CLIP
image / text towers (decord, clip) are the frozen front end and stay outside: the caller passes
features and a ``clip_model`` object with ``encode_text`` (plus an optional ``tokenize``).
"""
from __future__ import annotations

from typing import List, Sequence

import torch

from .. import engine
from .._lib import lib, check, SIM_BF16X3
from .validate import time_process

GRID_TOKENS = 18 * 18   # inference.py:59: the middle tokens of one frame (an 18 x 18 grid)
POOLED_TOKENS = 16      # inference.py:59: pooled to 16 tokens per frame


def adaptive_avg_pool2d(x: torch.Tensor, output_size) -> torch.Tensor:
    """F.adaptive_avg_pool2d(x, output_size) for fp32 x [..., H, W] on the K2 kernel."""
    oh, ow = int(output_size[0]), int(output_size[1])
    x = x.detach().float()
    *lead, H, W = x.shape
    if x.stride(-1) != 1:
        x = x.contiguous()
    planes = x.reshape(-1, H, W) if x.dim() != 3 else x
    if planes.stride(-1) != 1 or (planes.shape[0] > 1 and planes.stride(0) < (H - 1) * planes.stride(1) + W):
        planes = planes.contiguous()
    P = planes.shape[0]
    out = torch.empty((P, oh, ow), dtype=torch.float32, device=x.device)
    if P:
        check(lib.cmve_adaptive_avg_pool2d(engine.handle(x.device), engine._ptr(planes), P, H, W,
                                           planes.stride(0) if P > 1 else H * planes.stride(1), planes.stride(1),
                                           oh, ow, engine._ptr(out)), "cmve_adaptive_avg_pool2d")
    return out.view(*lead, oh, ow)


def _encode_text(clip_model, mod_text, tokenize, dev):
    if tokenize is None:
        import clip  # OpenAI CLIP tokenizer; not installed in the build image
        tokenize = clip.tokenize
    return clip_model.encode_text(tokenize(mod_text).to(dev))


@torch.no_grad()
def compute_cirr_val_metrics(ref_vdo_feature, mod_text, clip_model, index_features: torch.Tensor,
                             index_names: List[str], combining_function, combiner, tokenize=None):
    """inference.py:26-66 (same signature + optional tokenizer): the top-1 index name."""
    dev = index_features.device if torch.is_tensor(index_features) else engine.default_device()
    high, middle = ref_vdo_feature
    high = torch.as_tensor(high).to(dev).float().unsqueeze(0)                    # [1, T, D]
    middle = torch.as_tensor(middle).to(dev).float()                             # [T, 324, C]
    d = index_features.shape[-1]
    middle = adaptive_avg_pool2d(middle.reshape(1, middle.shape[0], GRID_TOKENS, -1), (POOLED_TOKENS, d))
    text = _encode_text(clip_model, mod_text, tokenize, dev)
    pred = combining_function((high, middle), text)                             # [1, D]
    gallery = engine.RowSet(torch.as_tensor(index_features).to(dev).float(), eps=1e-12, with_lo=True, device=dev)
    # argmin of 1 - pred . g == argmax of the cosine (pred is unit-norm from the combiner; a scale does
    # not change the order): the exact top-1
    q = engine.RowSet(pred.float(), eps=1e-12, with_lo=True, device=dev)
    idx, _ = engine.topk(q, gallery, 1, mode=SIM_BF16X3)
    return index_names[int(idx[0][0])]


@torch.no_grad()
def retrieve_top1(ref_vdo_feature, mod_text, clip_model, target_features: Sequence[torch.Tensor],
                  tar_list: List[str], combining_function, combiner, tokenize=None):
    """inference.py:124-136 from features: index_features = concat(time_process(high[None])) over the
    target videos (here one K2 launch over the stacked [N, T, D] highs), then the top-1 name."""
    feats = torch.stack([torch.as_tensor(t).float() for t in target_features])
    index_features = combiner.time_process(feats.to(engine.default_device()))
    return compute_cirr_val_metrics(ref_vdo_feature, mod_text, clip_model, index_features, tar_list,
                                    combining_function, combiner, tokenize)
