"""C5 end to end (BASELINE configs[4]): MCT's TSN feature extraction feeding the
retrieval gallery, on libcmve.so.

  tsn_feature_extraction(x, batches)   MCT/mmaction/models/recognizers/recognizer2d.py:76-83
        (Recognizer2D with test_cfg feature_extraction=True, configs/recognition/tsn/
        tsn_r50_clip_feature_extraction_1x1x3_rgb.py: 25 segments of a ResNet-50): the backbone's
        maps [batches * num_segs, C, H, W] -> AdaptiveAvgPool2d(1) -> reshape (batches, num_segs, C)
        -> mean over the segments, on K2 (``cmve_tsn_pool``).
  TSNGallery                           the chain the reference leaves to the user between MCT's
        extracted features and LINAS's retrieval: segment features -> K2 pool -> projection head
        (a LINAS ``Latent_mapping`` 2048 -> 1024: fc + BN-eval + l2norm on K3 / K1, or an ``nn.Linear``)
        -> rows of a resident gallery shard, packed once (fp16 + bf16 planes, fp64 norms, error bounds)
        -> exact ranks / exact top-k through ``cmve.dist.ShardedGallery`` (one shard per GPU).
The ResNet-50 backbone itself is a frozen PyTorch-ROCm module (out of scope); the
reference ships no MCT checkpoint, so the head weights are the caller's (seeded in tests and bench).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from . import engine
from . import _lib
from .dist import ShardedGallery
from .linas import model as LM


def tsn_feature_extraction(x: torch.Tensor, batches: int) -> torch.Tensor:
    """recognizer2d.py:76-83 on K2: x [batches * num_segs, C, H, W] (or [batches * num_segs, C] /
    [batches, num_segs, C] maps already pooled spatially) fp32 device -> [batches, C]."""
    x = x.detach()
    if not x.is_cuda:
        raise RuntimeError("tsn_feature_extraction expects a device tensor (no CPU fallback)")
    if x.dim() == 3 and x.shape[0] == batches:      # [B, S, C]
        x = x.reshape(-1, x.shape[2])
    if x.dim() == 2:
        x = x[:, :, None, None]
    if x.dim() != 4 or x.shape[0] % batches:
        raise ValueError(f"tsn_feature_extraction: maps {tuple(x.shape)} do not split into {batches} videos")
    n, C, H, W = x.shape
    S = n // batches
    x = x.to(torch.float32).contiguous()
    out = torch.empty((batches, C), dtype=torch.float32, device=x.device)
    for b0 in range(0, batches, 65535):  # grid.y limit per call
        nb = min(65535, batches - b0)
        _lib.check(_lib.lib.cmve_tsn_pool(engine.handle(x.device), engine._ptr(x[b0 * S:(b0 + nb) * S]), nb, S, C,
                                          H * W, engine._ptr(out[b0:b0 + nb]), out.stride(0)), "cmve_tsn_pool")
    return out


class TSNGallery:
    """A gallery shard built from TSN segment features: ``ingest`` chunks of videos (any order of calls,
    each writing its rows at the next free position), then ``finalize`` packs the shard once and returns
    the ``ShardedGallery`` that ranks / top-ks against it.

    head: ``cmve.linas.model.Latent_mapping`` (eval: fc + BN + l2norm on the split-bf16 GEMM kernel) or an
    ``nn.Linear`` (the pack normalises its rows, as the reference's cal_error does).  n_videos: this
    shard's capacity; offset / n_global / comm: its place in a sharded gallery (defaults: one shard)."""

    def __init__(self, n_videos: int, head: nn.Module, offset: int = 0, n_global: Optional[int] = None,
                 comm=None, device: Optional[torch.device] = None):
        self.device = device or engine.default_device()
        self.head = head.to(self.device).eval()
        dim = head.out_features if isinstance(head, nn.Linear) else self._mapping_out(head)
        self.rows = torch.empty((int(n_videos), dim), dtype=torch.float32, device=self.device)
        self.n = 0
        self.offset, self.n_global, self.comm = int(offset), n_global, comm
        self._packed = LM._PackedWeight()

    @staticmethod
    def _mapping_out(head):
        fcs = [m for m in head.modules() if isinstance(m, nn.Linear)]
        if not fcs:
            raise TypeError("TSNGallery: the head needs a Linear layer")
        return fcs[-1].out_features

    @torch.no_grad()
    def project(self, pooled: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The projection head on pooled [b, C] features (into `out` when given)."""
        if isinstance(self.head, nn.Linear):
            return LM.linear_fused(pooled, self.head.weight, self.head.bias, packed=self._packed, out=out)
        y = self.head(pooled)
        if out is not None:
            out.copy_(y)
            return out
        return y

    @torch.no_grad()
    def ingest(self, x: torch.Tensor, batches: int) -> slice:
        """Pool + project `batches` videos' segment maps (see tsn_feature_extraction) into the next rows;
        returns the rows' slice."""
        if self.n + batches > self.rows.shape[0]:
            raise ValueError(f"TSNGallery.ingest: {self.n} + {batches} videos exceed the capacity "
                             f"{self.rows.shape[0]}")
        pooled = tsn_feature_extraction(x, batches)
        sl = slice(self.n, self.n + batches)
        self.project(pooled, out=self.rows[sl])
        self.n += batches
        return sl

    def reset(self):
        """Forget the ingested rows (the buffer is kept): the next ingest writes row 0 again."""
        self.n = 0

    def finalize(self, with_lo: bool = False, **kw) -> ShardedGallery:
        """Pack the ingested rows once (resident in HBM) as this rank's gallery shard."""
        n_global = self.n_global if self.n_global is not None else self.offset + self.n
        return ShardedGallery(self.rows[:self.n], offset=self.offset, n_global=n_global, with_lo=with_lo,
                              device=self.device, comm=self.comm, **kw)
