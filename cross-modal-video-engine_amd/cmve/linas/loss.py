"""Mirror of ``LINAS-engine/loss.py`` (TripletLoss + cosine_sim) on libcmve.so, with autograd.

``TripletLoss(margin, measure, max_violation, cost_style, direction).forward(s, im)`` keeps the
reference's signature and semantics (loss.py:83-153): s = caption embeddings, im = video
embeddings, S = im . s^T (cosine_sim, loss.py:7-10).  Forward and backward are HIP kernels
(K6, fp32 S by ``cmve_gemm_f32``); only the cosine measure is on the MI355X path.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import engine
from .._lib import lib, check, PW_SQ_L2, PW_L1, PW_ORDER, PW_JACCARD


def _h(t):
    return engine.handle(t.device)


def gemm_f32(a: torch.Tensor, b: torch.Tensor, trans_a=False, trans_b=False, alpha=1.0) -> torch.Tensor:
    """alpha * op(a) @ op(b) in fp32 on the HIP GEMM (row-major, contiguous inputs)."""
    a = a.contiguous().float()
    b = b.contiguous().float()
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    N = b.shape[0] if trans_b else b.shape[1]
    out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    check(lib.cmve_gemm_f32(_h(a), int(trans_a), int(trans_b), M, N, K, float(alpha), engine._ptr(a), a.stride(0),
                            engine._ptr(b), b.stride(0), 0.0, engine._ptr(out), out.stride(0)), "cmve_gemm_f32")
    return out


def cosine_sim(im, s):
    """loss.py:7-10: im.mm(s.t())."""
    return gemm_f32(im, s, trans_b=True)


# ---- non-cosine similarities (loss.py:13-73) on the K10 all-pairs kernel: score[i_im, j_s] ----
# forward only: a caller that needs their gradient gets an error, not a silently detached result
def _pw(im, s, metric, alpha, beta):
    if torch.is_grad_enabled() and (im.requires_grad or s.requires_grad):
        raise NotImplementedError("cmve: the non-cosine similarities are forward-only (evaluation); their "
                                  "backward is not on the MI355X path")
    dev = im.device if im.is_cuda else engine.default_device()
    a = engine.to_device(im, dev, torch.float32)
    b = engine.to_device(s, dev, torch.float32)
    return engine.pairwise(a, b, metric, alpha, beta, torch.float32)


def order_sim(im, s):
    """loss.py:13-19: -sqrt(sum max(0, s_j - im_i)^2)."""
    return _pw(im, s, PW_ORDER, -1.0, 0.0)


def euclidean_sim(im, s):
    """loss.py:22-28: -sum (s_j - im_i)^2 (squared, as the reference)."""
    return _pw(im, s, PW_SQ_L2, -1.0, 0.0)


def L1_sim(im, s):
    """loss.py:31-37."""
    return _pw(im, s, PW_L1, -1.0, 0.0)


def L1_sim_norm(im, s):
    """loss.py:39-45: L1 / D - 1."""
    return _pw(im, s, PW_L1, 1.0 / im.shape[1], -1.0)


def L2_sim(im, s):
    """loss.py:48-54: -sum (s_j - im_i)^2."""
    return _pw(im, s, PW_SQ_L2, -1.0, 0.0)


def L2_sim_norm(im, s):
    """loss.py:56-62: sum (s_j - im_i)^2 / D - 1."""
    return _pw(im, s, PW_SQ_L2, 1.0 / im.shape[1], -1.0)


def jaccard_sim(im, s):
    """loss.py:65-73: sum min / sum max."""
    return _pw(im, s, PW_JACCARD, 1.0, 0.0)


_DIRS = {"v2t": 1, "t2v": 2, "all": 3}


class _TripletFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, im, margin, max_violation, dirs, mean_style):
        S = cosine_sim(im.detach(), s.detach())
        B = S.shape[0]
        dev = S.device
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        rv = torch.empty(B, dtype=torch.float32, device=dev)
        ra = torch.empty(B, dtype=torch.int32, device=dev)
        cv = torch.empty(B, dtype=torch.float32, device=dev)
        ca = torch.empty(B, dtype=torch.int32, device=dev)
        check(lib.cmve_triplet_fwd(_h(S), engine._ptr(S), S.stride(0), B, float(margin), int(max_violation), dirs,
                                   int(mean_style), engine._ptr(loss), engine._ptr(rv), engine._ptr(ra),
                                   engine._ptr(cv), engine._ptr(ca)), "cmve_triplet_fwd")
        ctx.save_for_backward(s.detach(), im.detach(), S, ra, ca)
        ctx.cfg = (float(margin), int(max_violation), dirs, int(mean_style))
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        s, im, S, ra, ca = ctx.saved_tensors
        margin, mv, dirs, mean_style = ctx.cfg
        B = S.shape[0]
        g = g.reshape(1).float().contiguous()
        dS = torch.empty_like(S)
        check(lib.cmve_triplet_bwd(_h(S), engine._ptr(S), S.stride(0), B, margin, mv, dirs, mean_style,
                                   engine._ptr(g), engine._ptr(ra), engine._ptr(ca), engine._ptr(dS), dS.stride(0)),
              "cmve_triplet_bwd")
        d_im = gemm_f32(dS, s)                 # dL/dim = dS . s
        d_s = gemm_f32(dS, im, trans_a=True)   # dL/ds  = dS^T . im
        return d_s.to(s.dtype), d_im.to(im.dtype), None, None, None, None


class TripletLoss(nn.Module):
    """loss.py:83-153 -- triplet ranking loss (cosine measure)."""

    def __init__(self, margin=0, measure=False, max_violation=False, cost_style='sum', direction='all'):
        super().__init__()
        if measure not in (False, None, 'cosine'):
            raise NotImplementedError(f"cmve TripletLoss: measure {measure!r} not on the MI355X path (cosine only)")
        self.margin = margin
        self.cost_style = cost_style
        self.direction = direction
        self.max_violation = max_violation

    def forward(self, s, im):
        if self.direction not in _DIRS:
            # the reference falls through to Variable(torch.zeros(1)) for both terms (loss.py:145-148)
            return torch.zeros((), device=s.device)
        return _TripletFn.apply(s, im, self.margin, self.max_violation, _DIRS[self.direction],
                                self.cost_style != 'sum')


NAME_TO_SIM = {'cosine': cosine_sim, 'order': order_sim, 'euclidean': euclidean_sim, 'jaccard': jaccard_sim}


def get_sim(name):
    assert name in NAME_TO_SIM, '%s not supported.' % name
    return NAME_TO_SIM[name]
