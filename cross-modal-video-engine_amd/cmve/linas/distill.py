"""Distillation losses and the 'distill_from_best_model' training step of LINAS on libcmve.so
(SURVEY 8f rank 3).

  MSELoss / SmoothL1Loss / KLDivLoss (sum | mean)      model.py:554-580  (K15 cmve_pair_loss_*)
  similarity_distill_loss(vid, cap, s_vid, s_cap)      model.py:845-878  forward_loss_distill_similarity:
      s1 = vid . cap^T (teacher, detached), s2 = s_vid . s_cap^T (fp32 MFMA GEMM, cmve_gemm_f32), then
      SmoothL1(s1, s2) -- or its 'diag' / 'adapt' weighted sums, 'maxdiag' = -trace(s2), 'svd'
      (log singular values: torch.svd of the B x B matrices on the host, as the reference, because its
      a.diag(log b).c with c = V, not V^T, depends on the SVD library's sign convention)
  distill_loss(student, teacher, distill_type, ...)    model.py:880-889  forward_loss_distill
  DistillTrainer.train_emb                             model.py:916-982  train_emb, style
      'distill_from_best_model': student 'text+video' (no optimizer.zero_grad() in that branch:
      gradients accumulate across steps, reproduced) and 'map' / 'de+map' (with_detach, finetune_vid)

The trainer drives the projection heads (Latent_mapping on the K3 / K11 functions of
cmve.linas.train); the encoders are the frozen backbones, so its inputs are encoder features (or
optional encoder callables), as GTTrainer's.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import engine
from .._lib import lib, check, PAIR_MSE, PAIR_SMOOTH_L1, PAIR_KL
from .loss import gemm_f32, TripletLoss
from .train import Adam, clip_grad_norm_

_p = engine._ptr


def _f32c(t):
    t = t.detach()
    t = t if t.dtype == torch.float32 else t.float()
    return t if t.is_contiguous() else t.contiguous()


class _PairLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y, w, kind, scale):
        xs, ys = _f32c(x), _f32c(y)
        ws = _f32c(w) if w is not None else None
        if xs.shape != ys.shape or (ws is not None and ws.shape != xs.shape):
            raise ValueError("cmve pair loss: input / target / weight shapes differ")
        loss = torch.empty((), dtype=torch.float32, device=xs.device)
        check(lib.cmve_pair_loss_fwd(engine.handle(xs.device), _p(xs), _p(ys), _p(ws), xs.numel(), kind, scale,
                                     _p(loss)), "cmve_pair_loss_fwd")
        ctx.save_for_backward(xs, ys, ws)
        ctx.kind, ctx.scale = kind, scale
        return loss

    @staticmethod
    def backward(ctx, g):
        xs, ys, ws = ctx.saved_tensors
        gx = torch.empty_like(xs) if ctx.needs_input_grad[0] else None
        gy = torch.empty_like(ys) if ctx.needs_input_grad[1] else None
        gg = _f32c(g).reshape(1)
        check(lib.cmve_pair_loss_bwd(engine.handle(xs.device), _p(xs), _p(ys), _p(ws), xs.numel(), ctx.kind, ctx.scale,
                                     _p(gg), _p(gx), _p(gy)), "cmve_pair_loss_bwd")
        return gx, gy, None, None, None


def pair_loss(x, y, kind, scale=1.0, weight=None):
    """scale * sum_i w_i f(x_i, y_i) as a 0-d device tensor with autograd (K15)."""
    return _PairLossFn.apply(x, y, weight, int(kind), float(scale))


def _reduction(size_average=None, reduce=None, reduction="mean"):
    if size_average is not None or reduce is not None:  # torch's legacy arguments (model.py:554-580)
        size_average = True if size_average is None else size_average
        reduce = True if reduce is None else reduce
        reduction = "none" if not reduce else ("mean" if size_average else "sum")
    if reduction not in ("sum", "mean"):
        raise NotImplementedError("cmve pair losses: reduction 'sum' or 'mean' (the elementwise 'none' criteria of "
                                  "model.py:555-556 are the weighted sums of similarity_distill_loss)")
    return reduction


class _PairLoss(nn.Module):
    kind = PAIR_MSE

    def __init__(self, size_average=None, reduce=None, reduction="mean"):
        super().__init__()
        self.reduction = _reduction(size_average, reduce, reduction)

    def forward(self, input, target):
        scale = 1.0 / input.numel() if self.reduction == "mean" and input.numel() else 1.0
        return pair_loss(input, target, self.kind, scale)


class MSELoss(_PairLoss):
    """nn.MSELoss (model.py:554,557,560)."""
    kind = PAIR_MSE


class SmoothL1Loss(_PairLoss):
    """nn.SmoothL1Loss, beta 1 (model.py:555,578,580)."""
    kind = PAIR_SMOOTH_L1


class KLDivLoss(_PairLoss):
    """nn.KLDivLoss(input, target), log_target False; 'mean' divides by every element, as torch's
    legacy size_average (model.py:558,561)."""
    kind = PAIR_KL


class _SimFn(torch.autograd.Function):
    """S = A . B^T (forward_loss_distill_similarity's s2) on the exact-fp32 MFMA GEMM."""

    @staticmethod
    def forward(ctx, a, b):
        a32, b32 = _f32c(a), _f32c(b)
        ctx.save_for_backward(a32, b32)
        return gemm_f32(a32, b32, trans_b=True)

    @staticmethod
    def backward(ctx, dS):
        a32, b32 = ctx.saved_tensors
        dS = _f32c(dS)
        da = gemm_f32(dS, b32) if ctx.needs_input_grad[0] else None
        db = gemm_f32(dS, a32, trans_a=True) if ctx.needs_input_grad[1] else None
        return da, db


def sim(a, b):
    return _SimFn.apply(a, b)


def _log_svd(s):
    """model.py:848-851: a . diag(log b) . c with c = V (not V^T), reproduced.  That product pairs
    column i of U with ROW i of V, so it depends on the SVD's per-vector sign convention: the B x B
    decomposition runs where the reference's does (LAPACK, host) and the result returns to the device,
    autograd included.  A device SVD (rocSOLVER) flips other signs and gives another loss."""
    a, b, c = torch.svd(s.cpu())
    return torch.matmul(a, torch.matmul(torch.diag(torch.log(b)), c)).to(s.device)


def similarity_distill_loss(vid_emb, cap_emb, student_vid_emb, student_cap_emb, similarity_type=None,
                            cost_style="sum", mask=None):
    """forward_loss_distill_similarity (model.py:845-878); vid_emb / cap_emb are the teacher's
    (detached by the caller, model.py:931)."""
    s1 = gemm_f32(_f32c(vid_emb), _f32c(cap_emb), trans_b=True)
    s2 = sim(student_vid_emb, student_cap_emb)
    B = s1.shape[0]
    mean = 1.0 / s1.numel() if cost_style == "mean" else 1.0
    if similarity_type == "svd":
        return pair_loss(_log_svd(s2), _log_svd(s1), PAIR_SMOOTH_L1, mean)
    if similarity_type == "eig":
        raise NotImplementedError("similarity_type 'eig' calls torch.eig (model.py:853-857), removed from torch")
    if similarity_type == "diag":   # sum(diagonal(huber(s1, s2)))
        return pair_loss(s2, s1, PAIR_SMOOTH_L1, 1.0, torch.eye(B, device=s1.device))
    if similarity_type == "adapt":  # sum(softmax(mask, 0) * huber(s1, s2)) * batchsize
        if mask is None:
            raise ValueError("similarity_type 'adapt' needs the model's mask (model.py:586-588)")
        w = F.softmax(mask.detach().float(), dim=0)
        return pair_loss(s2, s1, PAIR_SMOOTH_L1, float(mask.shape[0]), w)
    if similarity_type == "maxdiag":
        return -torch.sum(torch.diagonal(s2))
    return pair_loss(s2, s1, PAIR_SMOOTH_L1, mean)   # similarity_loss = SmoothL1Loss(sum | mean)


def distill_loss(student, teacher, distill_type, cost_style="sum"):
    """forward_loss_distill (model.py:880-889): 'mse', 'kl' or 'mse+kl' (distill_criterion /
    distill_kl with the cost_style reduction)."""
    red = "mean" if cost_style == "mean" else "sum"
    if distill_type == "mse":
        return MSELoss(reduction=red)(student, teacher)
    if distill_type == "kl":
        return KLDivLoss(reduction=red)(student, teacher)
    if distill_type == "mse+kl":
        return MSELoss(reduction=red)(student, teacher) + KLDivLoss(reduction=red)(student, teacher)
    raise ValueError(f"distill_type {distill_type!r}: the reference computes no loss for it (model.py:880-887)")


class DistillTrainer:
    """train_emb for style 'distill_from_best_model' (model.py:916-982) around the HIP heads.

    Modules follow Dual_Encoding's names; the parameter list and its order follow init_info
    (model.py:481-494): vid_mapping, text_mapping, student_text_mapping, student_vid_mapping (plus the
    optional encoder modules first).  ``videos`` / ``captions`` are encoder features: for
    'text+video' a pair (teacher features, student features) each; otherwise captions is
    (teacher text features, student text features) and videos the teacher video features."""

    def __init__(self, vid_mapping, text_mapping, student_text_mapping, student_vid_mapping=None,
                 criterion: Optional[nn.Module] = None, student_model="text+video", distill_loss="text+video",
                 distill_type="mse", cost_style="sum", alpha=1.0, beta=1.0, video_alpha=1.0,
                 distill_with_triplet=True, distill_with_similarity=False, similarity_type=None,
                 with_detach=False, finetune_vid=False, learning_rate=1e-4, grad_clip=2.0, mask=None,
                 encoders=()):
        self.vid_mapping, self.text_mapping = vid_mapping, text_mapping
        self.student_text_mapping, self.student_vid_mapping = student_text_mapping, student_vid_mapping
        self.criterion = criterion if criterion is not None else TripletLoss(0.2, "cosine", True, cost_style, "all")
        self.student_model, self.distill_loss, self.distill_type = student_model, distill_loss, distill_type
        self.cost_style, self.alpha, self.beta, self.video_alpha = cost_style, alpha, beta, video_alpha
        self.distill_with_triplet, self.distill_with_similarity = distill_with_triplet, distill_with_similarity
        self.similarity_type, self.with_detach, self.finetune_vid = similarity_type, with_detach, finetune_vid
        self.grad_clip, self.mask = grad_clip, mask
        params = []
        for m in list(encoders) + [vid_mapping, text_mapping, student_text_mapping, student_vid_mapping]:
            if m is not None:
                params += list(m.parameters())
        self.params = params
        self.optimizer = Adam(self.params, lr=learning_rate)
        self.Eiters = 0

    def train_start(self):
        for m in (self.vid_mapping, self.text_mapping, self.student_text_mapping, self.student_vid_mapping):
            if m is not None:
                m.train()

    def forward_emb(self, videos, captions):
        """model.py:677-698 on encoder features."""
        if self.student_model == "text+video":
            (v, sv), (c, sc) = videos, captions
            return (self.vid_mapping(v), self.text_mapping(c), self.student_vid_mapping(sv),
                    self.student_text_mapping(sc))
        c, sc = captions
        return self.vid_mapping(videos), self.text_mapping(c), self.student_text_mapping(sc)

    def _distill(self, student, teacher):
        return distill_loss(student, teacher, self.distill_type, self.cost_style)

    def _clip_step(self, loss):
        loss.backward()
        coef = None
        if self.grad_clip > 0:
            _, coef = clip_grad_norm_(self.params, self.grad_clip, _apply=False)
        self.optimizer.step(grad_scale=coef)

    def train_emb(self, videos, captions):
        """One step; returns the reference's tuple (batch size, loss values ...)."""
        self.Eiters += 1
        red = "mean" if self.cost_style == "mean" else "sum"
        if self.student_model == "text+video":
            vid_emb, cap_emb, s_vid, s_cap = self.forward_emb(videos, captions)
            if self.distill_loss == "text+video":
                if self.distill_type == "cross":
                    loss1 = MSELoss(reduction=red)(s_cap, cap_emb.detach()) + \
                        KLDivLoss(reduction=red)(s_vid, vid_emb.detach())
                else:
                    loss1 = self._distill(s_cap, cap_emb.detach()) + \
                        self.video_alpha * self._distill(s_vid, vid_emb.detach())
            elif self.distill_loss == "text":
                loss1 = self._distill(s_cap, cap_emb.detach())
            elif self.distill_loss == "video":
                loss1 = self._distill(s_vid, vid_emb.detach())
            else:
                raise ValueError(f"distill_loss {self.distill_loss!r}")
            loss2 = self.criterion(s_cap, s_vid) if self.distill_with_triplet else None
            loss3 = (similarity_distill_loss(vid_emb.detach(), cap_emb.detach(), s_vid, s_cap, self.similarity_type,
                                             self.cost_style, self.mask) if self.distill_with_similarity else None)
            loss = self.alpha * loss1
            if loss2 is not None:
                loss = loss + loss2
            if loss3 is not None:
                loss = loss + self.beta * loss3
            # model.py:938-952: no optimizer.zero_grad() in this branch -- gradients accumulate
            self._clip_step(loss)
            return (vid_emb.size(0), loss1.item()) + tuple(x.item() for x in (loss2, loss3) if x is not None)
        vid_emb, cap_emb, s_cap = self.forward_emb(videos, captions)
        self.optimizer.zero_grad()
        loss2 = self._distill(s_cap, cap_emb.detach() if self.with_detach else cap_emb)
        value2 = loss2.item()
        if self.distill_with_triplet:
            v = vid_emb.detach() if (self.with_detach and not self.finetune_vid) else vid_emb
            loss3 = self.criterion(s_cap, v)
            value3 = loss3.item()
            loss = self.alpha * loss2 + loss3
        else:
            loss = self.alpha * loss2
        self._clip_step(loss)
        return (vid_emb.size(0), value2, value3) if self.distill_with_triplet else (vid_emb.size(0), value2)
