"""CPU oracle for the training-step row.

TEST INFRASTRUCTURE ONLY (see oracle/retrieval.py).  A numpy fp64 restatement of one 'GT'
training step of the LINAS heads, forward and hand-written backward:

  MFC training forward (LINAS-engine/model.py:97-116): fc1, residual relu blocks, BatchNorm1d
    with batch statistics (torch semantics: biased variance normalises, unbiased variance and
    momentum 0.1 update the running stats), dropout p = 0
  Latent_mapping l2norm (model.py:35-40, 374-381)
  TripletLoss (loss.py:83-153) via oracle.heads.triplet_loss
  clip_grad_norm_ (model.py:1000-1001) and torch.optim.Adam (model.py:593)

Pinned against tests/golden/train_step.npz and train_bn_l2.npz, produced by the reference's own
modules (tests/golden/make_golden_train.py; tests/test_train.py).
"""
from __future__ import annotations

import numpy as np

from oracle.heads import triplet_loss


def _f64(a):
    return np.asarray(a, np.float64)


def mapping_forward(x, P, n_lin, bn_eps=1e-5):
    """P: {'fc{k}.weight', 'fc{k}.bias', 'bn.weight', 'bn.bias'} -> (y, tape)."""
    x = _f64(x)
    tape = {"x": x}
    f = x @ _f64(P["fc1.weight"]).T + _f64(P["fc1.bias"])
    for k in range(2, n_lin + 1):
        z = f @ _f64(P[f"fc{k}.weight"]).T + _f64(P[f"fc{k}.bias"])
        tape[f"f{k - 1}"], tape[f"z{k}"] = f, z
        f = f + np.maximum(z, 0.0)
    tape[f"f{n_lin}"] = f
    mean = f.mean(0)
    var = f.var(0)  # biased
    inv = 1.0 / np.sqrt(var + bn_eps)
    xhat = (f - mean) * inv
    h = xhat * _f64(P["bn.weight"]) + _f64(P["bn.bias"])
    nrm = np.sqrt((h * h).sum(1, keepdims=True))
    tape.update(mean=mean, var=var, inv=inv, xhat=xhat, h=h, nrm=nrm)
    return h / nrm, tape


def mapping_backward(dy, P, n_lin, tape):
    """-> (dx, grads{name: array})."""
    h, nrm = tape["h"], tape["nrm"]
    dh = dy / nrm - h * ((h * dy).sum(1, keepdims=True) / nrm ** 3)
    xhat, inv = tape["xhat"], tape["inv"]
    g = {"bn.weight": (dh * xhat).sum(0), "bn.bias": dh.sum(0)}
    dxh = dh * _f64(P["bn.weight"])
    df = inv * (dxh - dxh.mean(0) - xhat * (dxh * xhat).mean(0))
    for k in range(n_lin, 1, -1):
        z, fprev = tape[f"z{k}"], tape[f"f{k - 1}"]
        dz = df * (z > 0)
        g[f"fc{k}.weight"] = dz.T @ fprev
        g[f"fc{k}.bias"] = dz.sum(0)
        df = df + dz @ _f64(P[f"fc{k}.weight"])
    g["fc1.weight"] = df.T @ tape["x"]
    g["fc1.bias"] = df.sum(0)
    dx = df @ _f64(P["fc1.weight"])
    return dx, g


def bn_running_update(rm, rv, tape, n, momentum=0.1):
    return ((1 - momentum) * _f64(rm) + momentum * tape["mean"],
            (1 - momentum) * _f64(rv) + momentum * tape["var"] * n / (n - 1))


def clip_grads(grads, max_norm):
    """clip_grad_norm_: total 2-norm over all grads; grads *= min(1, max_norm / (total + 1e-6))."""
    total = np.sqrt(sum(float((g * g).sum()) for g in grads))
    coef = min(1.0, max_norm / (total + 1e-6))
    return [g * coef for g in grads], total


def adam(p, g, m, v, step, lr, b1=0.9, b2=0.999, eps=1e-8):
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    return p - (lr / bc1) * m / (np.sqrt(v) / np.sqrt(bc2) + eps), m, v


class GTStep:
    """train_emb 'GT' (model.py:984-1004) over two heads: video P_v (n_lin_v), text P_t (n_lin_t)."""

    ORDER = ["fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias", "fc3.weight", "fc3.bias", "fc4.weight",
             "fc4.bias", "bn.weight", "bn.bias"]

    def __init__(self, P_v, n_lin_v, run_v, P_t, n_lin_t, run_t, lr, grad_clip, margin=0.2):
        self.heads = [[{k: _f64(v) for k, v in P_v.items()}, n_lin_v, [_f64(r) for r in run_v]],
                      [{k: _f64(v) for k, v in P_t.items()}, n_lin_t, [_f64(r) for r in run_t]]]
        self.lr, self.grad_clip, self.margin = lr, grad_clip, margin
        self.names = [[k for k in self.ORDER if k in h[0]] for h in self.heads]  # nn.Module parameter order
        self.m = [[np.zeros_like(h[0][k]) for k in names] for h, names in zip(self.heads, self.names)]
        self.v = [[np.zeros_like(h[0][k]) for k in names] for h, names in zip(self.heads, self.names)]
        self.t = 0

    def step(self, videos, captions):
        (Pv, nv, rv), (Pt, nt, rt) = self.heads
        vid, tv = mapping_forward(videos, Pv, nv)
        cap, tt = mapping_forward(captions, Pt, nt)
        loss, d_cap, d_vid = triplet_loss(cap, vid, self.margin, True, False, 3)
        _, gv = mapping_backward(d_vid, Pv, nv, tv)
        _, gt = mapping_backward(d_cap, Pt, nt, tt)
        n = vid.shape[0]
        rv[0], rv[1] = bn_running_update(rv[0], rv[1], tv, n)
        rt[0], rt[1] = bn_running_update(rt[0], rt[1], tt, n)
        flat = [gv[k] for k in self.names[0]] + [gt[k] for k in self.names[1]]
        total = np.sqrt(sum(float((g * g).sum()) for g in flat))
        if self.grad_clip > 0:
            flat, total = clip_grads(flat, self.grad_clip)
        self.t += 1
        i = 0
        for hi, (h, names) in enumerate(zip(self.heads, self.names)):
            for j, k in enumerate(names):
                h[0][k], self.m[hi][j], self.v[hi][j] = adam(h[0][k], flat[i], self.m[hi][j], self.v[hi][j],
                                                             self.t, self.lr)
                i += 1
        return loss, total, flat, vid, cap
