"""Bidirectional InfoNCE on libcmve.so (K7), with autograd.

Row half  = ``nn.CrossEntropyLoss()(logits, arange(B))`` with ``logits = 100 * pred @ target.T``
            (MultiFusion/src/combiner.py:136, MultiFusion/src/combiner_train.py:318,367-372);
col half  = the same CE on ``logits.T`` (the transposed logits of
            MCT/mmaction/models/backbones/clip.py:383-386).
``direction='both'`` returns (row + col) / 2.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import engine
from .._lib import lib, check
from ..linas.loss import gemm_f32

_DIRS = {"row": 1, "col": 2, "both": 3}


class _InfoNCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, scale, dirs):
        S = gemm_f32(pred.detach(), target.detach(), trans_b=True)
        B = S.shape[0]
        dev = S.device
        loss3 = torch.empty(3, dtype=torch.float32, device=dev)
        rl = torch.empty(B, dtype=torch.float64, device=dev)
        cl = torch.empty(B, dtype=torch.float64, device=dev)
        rv = torch.empty(B, dtype=torch.float32, device=dev)
        cv = torch.empty(B, dtype=torch.float32, device=dev)
        check(lib.cmve_infonce_fwd(engine.handle(dev), engine._ptr(S), S.stride(0), B, float(scale), dirs,
                                   engine._ptr(loss3), engine._ptr(rl), engine._ptr(cl), engine._ptr(rv),
                                   engine._ptr(cv)), "cmve_infonce_fwd")
        ctx.save_for_backward(pred.detach(), target.detach(), S, rl, cl)
        ctx.cfg = (float(scale), dirs)
        return loss3[2]

    @staticmethod
    def backward(ctx, g):
        pred, target, S, rl, cl = ctx.saved_tensors
        scale, dirs = ctx.cfg
        B = S.shape[0]
        g = g.reshape(1).float().contiguous()
        dS = torch.empty_like(S)
        check(lib.cmve_infonce_bwd(engine.handle(S.device), engine._ptr(S), S.stride(0), B, scale, dirs,
                                   engine._ptr(g), engine._ptr(rl), engine._ptr(cl), engine._ptr(dS), dS.stride(0)),
              "cmve_infonce_bwd")
        d_pred = gemm_f32(dS, target)
        d_target = gemm_f32(dS, pred, trans_a=True)
        return d_pred.to(pred.dtype), d_target.to(target.dtype), None, None


class InfoNCE(nn.Module):
    def __init__(self, scale: float = 100.0, direction: str = "both"):
        super().__init__()
        if direction not in _DIRS:
            raise ValueError(f"InfoNCE direction must be one of {sorted(_DIRS)}")
        self.scale = scale
        self.direction = direction

    def forward(self, pred, target):
        """pred, target: [B, D] (already normalised, as combiner.py:133-136 feeds them)."""
        return _InfoNCEFn.apply(pred, target, self.scale, _DIRS[self.direction])
