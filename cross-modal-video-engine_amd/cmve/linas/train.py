"""Training step of the LINAS projection heads on libcmve.so.

``GTTrainer.train_emb`` mirrors ``LINAS-engine/model.py:984-1004`` (``train_emb``, style 'GT')::

    vid_emb, cap_emb = forward_emb(...)        # encoders (PyTorch, or pooled features) -> Latent_mapping (HIP)
    optimizer.zero_grad()
    loss = criterion(cap_emb, vid_emb)         # TripletLoss (K6) -- or InfoNCE (K7)
    loss.backward()                            # autograd through the K3 / gemm_f32 / K11 functions below
    clip_grad_norm_(params, grad_clip)         # K11: fp64 norm, coefficient computed on the device
    optimizer.step()                           # K11: Adam

The heads' training forward (``MFC.forward`` in training mode, model.py:97-116) is a chain of
autograd Functions, each a HIP kernel forward and backward:

    _LinearFn      z = x W^T + b      fwd/bwd on the exact-fp32 MFMA GEMM (cmve_gemm_f32[_ex]) + column sums
    _ResidReluFn   f + relu(z)        (model.py:104-109)
    _BatchNormFn   BatchNorm1d, batch statistics, running stats updated (model.py:111-112)
    _DropoutFn     nn.Dropout(p) with a counter-hash mask (same distribution, NOT torch's random stream)
    _L2NormFn      x / ||x||, no epsilon (model.py:35-40)

``Adam`` and ``clip_grad_norm_`` keep the torch.optim.Adam / torch.nn.utils.clip_grad_norm_
interfaces and update order; their arithmetic runs in K11 kernels with no host synchronisation.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from .. import engine
from .._lib import lib, check

_p = engine._ptr


def _h(t: torch.Tensor) -> int:
    return engine.handle(t.device)


def _f32(t: torch.Tensor) -> torch.Tensor:
    t = t.detach()
    if t.dtype != torch.float32:
        t = t.float()
    return t if t.is_contiguous() else t.contiguous()


# ---------------------------------------------------------------- autograd functions
class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        xs, w = _f32(x), _f32(weight)
        z = torch.empty((xs.shape[0], w.shape[0]), dtype=torch.float32, device=xs.device)
        b = _f32(bias) if bias is not None else None
        check(lib.cmve_gemm_f32_ex(_h(xs), 0, 1, xs.shape[0], w.shape[0], xs.shape[1], 1.0, _p(xs), xs.stride(0),
                                   _p(w), w.stride(0), 0.0, _p(z), z.stride(0), _p(b), 0), "cmve_gemm_f32_ex")
        ctx.save_for_backward(xs, w)
        ctx.has_bias = bias is not None
        return z

    @staticmethod
    def backward(ctx, dz):
        from .loss import gemm_f32
        x, w = ctx.saved_tensors
        dz = _f32(dz)
        dx = gemm_f32(dz, w) if ctx.needs_input_grad[0] else None                      # [n, K]   = dz . W
        dw = gemm_f32(dz, x, trans_a=True) if ctx.needs_input_grad[1] else None        # [F, K]   = dz^T . x
        db = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = torch.empty(dz.shape[1], dtype=torch.float32, device=dz.device)
            check(lib.cmve_col_sum(_h(dz), _p(dz), dz.stride(0), dz.shape[0], dz.shape[1], _p(db)), "cmve_col_sum")
        return dx, dw, db


class _ResidReluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feats, z):
        f, z = _f32(feats), _f32(z)
        out = torch.empty_like(z)
        check(lib.cmve_resid_relu(_h(z), _p(z), _p(f), z.numel(), _p(out)), "cmve_resid_relu")
        ctx.save_for_backward(z)
        return out

    @staticmethod
    def backward(ctx, dout):
        (z,) = ctx.saved_tensors
        dout = _f32(dout)
        dz = torch.empty_like(z)
        check(lib.cmve_relu_grad(_h(z), _p(z), _p(dout), z.numel(), _p(dz)), "cmve_relu_grad")
        return dout, dz


class _BatchNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, factor, eps):
        xs = _f32(x)
        n, d = xs.shape
        y = torch.empty_like(xs)
        smean = torch.empty(d, dtype=torch.float32, device=xs.device)
        sinv = torch.empty_like(smean)
        check(lib.cmve_bn_train_fwd(_h(xs), _p(xs), xs.stride(0), n, d, _p(weight), _p(bias), float(eps),
                                    float(factor), _p(running_mean), _p(running_var), _p(y), y.stride(0),
                                    _p(smean), _p(sinv)), "cmve_bn_train_fwd")
        ctx.save_for_backward(xs, weight.detach() if weight is not None else None)
        ctx.affine = (weight is not None, bias is not None)
        ctx.eps = float(eps)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = _f32(dy)
        n, d = x.shape
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty(d, dtype=torch.float32, device=x.device) if ctx.affine[0] else None
        db = torch.empty(d, dtype=torch.float32, device=x.device) if ctx.affine[1] else None
        check(lib.cmve_bn_train_bwd(_h(x), _p(dy), dy.stride(0), _p(x), x.stride(0), n, d, _p(w), ctx.eps,
                                    _p(dx), dx.stride(0) if dx is not None else d, _p(dw), _p(db)),
              "cmve_bn_train_bwd")
        return dx, dw, db, None, None, None, None


_DROPOUT = {"seed": 0x5EED, "counters": {}}


def _dropout_counter(device) -> torch.Tensor:
    """Per-device call counter of the dropout stream, kept ON the device so that graph replays
    draw fresh masks (each call advances it on the stream)."""
    c = _DROPOUT["counters"].get(device)
    if c is None:
        c = torch.zeros(1, dtype=torch.int64, device=device)
        _DROPOUT["counters"][device] = c
    return c


def manual_seed(seed: int):
    """Seed (and rewind) the training dropout masks (counter-hash stream; independent of torch's RNG)."""
    _DROPOUT["seed"] = int(seed) & ((1 << 64) - 1)
    for c in _DROPOUT["counters"].values():
        c.zero_()


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p):
        xs = _f32(x)
        n = xs.numel()
        y = torch.empty_like(xs)
        mask = torch.empty(xs.shape, dtype=torch.uint8, device=xs.device)
        counter = _dropout_counter(xs.device)  # a fresh 2^32-element window per call
        check(lib.cmve_dropout(_h(xs), _p(xs), n, float(p), _DROPOUT["seed"], 0, _p(y), _p(mask), _p(counter)),
              "cmve_dropout")
        ctx.save_for_backward(mask)
        ctx.scale = 1.0 / (1.0 - p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (mask,) = ctx.saved_tensors
        dy = _f32(dy)
        dx = torch.empty_like(dy)
        check(lib.cmve_mask_scale(_h(dy), _p(dy), _p(mask), dy.numel(), float(ctx.scale), _p(dx)), "cmve_mask_scale")
        return dx, None


class _L2NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        from .model import l2norm
        xs = _f32(x)
        ctx.save_for_backward(xs)
        return l2norm(xs)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = _f32(dy)
        dx = torch.empty_like(x)
        check(lib.cmve_l2norm_bwd(_h(x), _p(x), x.stride(0), _p(dy), dy.stride(0), x.shape[0], x.shape[1], _p(dx),
                                  dx.stride(0)), "cmve_l2norm_bwd")
        return dx


def linear(x, weight, bias=None):
    return _LinearFn.apply(x, weight, bias)


def resid_relu(feats, z):
    return _ResidReluFn.apply(feats, z)


def batch_norm_train(x, bn: nn.BatchNorm1d):
    """BatchNorm1d.forward in training mode (torch semantics, incl. num_batches_tracked / momentum None)."""
    factor = 0.0
    if bn.track_running_stats and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
        factor = (1.0 / float(bn.num_batches_tracked)) if bn.momentum is None else bn.momentum
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    return _BatchNormFn.apply(x, bn.weight, bn.bias, rm, rv, factor, bn.eps)


def dropout(x, p: float, training: bool = True):
    if not training or p == 0.0:
        return x
    return _DropoutFn.apply(x, float(p))


def l2norm_train(x):
    return _L2NormFn.apply(x)


def mfc_train_forward(mfc, inputs):
    """MFC.forward in training mode (model.py:97-116) on the functions above."""
    n_lin = min(mfc.n_fc, 5) - 1
    feats = linear(inputs, mfc.fc1.weight, mfc.fc1.bias)
    for k in range(2, n_lin + 1):
        fc = getattr(mfc, f"fc{k}")
        feats = resid_relu(feats, linear(feats, fc.weight, fc.bias))
    if mfc.have_bn and mfc.have_last_bn:
        feats = batch_norm_train(feats, mfc.bn_1)
    if mfc.have_dp:
        feats = dropout(feats, mfc.dropout.p, True)
    return feats


# ---------------------------------------------------------------- clip + Adam
def _ptr_array(ts):
    arr = (engine.C.c_void_p * max(1, len(ts)))(*[t.data_ptr() for t in ts])
    sizes = (engine.C.c_int64 * max(1, len(ts)))(*[t.numel() for t in ts])
    return arr, sizes


def _check_f32(ts, what):
    dev = ts[0].device
    for t in ts:
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device != dev:
            raise TypeError(f"cmve {what}: fp32 contiguous tensors on one device expected")


def clip_grad_norm_(parameters, max_norm: float, norm_type: float = 2.0, _apply: bool = True):
    """torch.nn.utils.clip_grad_norm_ (2-norm): grads *= min(1, max_norm / (||g|| + 1e-6)), in place;
    returns the total norm as a 0-d device tensor (no host synchronisation).  With _apply=False the
    grads are left alone and (total, coef) is returned, for Adam.step(grad_scale=coef) to apply."""
    if float(norm_type) != 2.0:
        raise NotImplementedError("cmve clip_grad_norm_: only the 2-norm (what model.py:1001 uses)")
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    grads = [p.grad for p in parameters if p.grad is not None]
    if not grads:
        return torch.tensor(0.0) if _apply else (torch.tensor(0.0), None)
    _check_f32(grads, "clip_grad_norm_")
    dev = grads[0].device
    out = torch.empty(2, dtype=torch.float32, device=dev)  # [total, coef]
    total, coef = out[0:1], out[1:2]
    ptrs, sizes = _ptr_array(grads)
    h = _h(grads[0])
    check(lib.cmve_grad_norm_multi(h, len(grads), ptrs, sizes, float(max_norm), _p(coef), _p(total)),
          "cmve_grad_norm_multi")
    if not _apply:
        return total[0], coef
    check(lib.cmve_scale_multi(h, len(grads), ptrs, sizes, _p(coef)), "cmve_scale_multi")
    return total[0]


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam (model.py:593); each param group's update is one multi-tensor K11 launch
    per 24 tensors.  State keys match torch's ('step' as a CPU float tensor, 'exp_avg', 'exp_avg_sq')."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False,
                 capturable=False):
        if amsgrad:
            raise NotImplementedError("cmve Adam: amsgrad is not on the MI355X path (model.py:593 does not use it)")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, capturable=capturable))

    @torch.no_grad()
    def step(self, closure=None, grad_scale: Optional[torch.Tensor] = None):
        """grad_scale: device f32[1] multiplying (and written back into) every grad first -- the
        deferred clip coefficient of clip_grad_norm_(..., _apply=False)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            _check_f32(ps + [p.grad for p in ps], "Adam")
            capturable = group.get("capturable", False)
            steps, dev_step = [], None
            if capturable:  # one device step counter per group, advanced on the stream (graph replays)
                if not all(p.grad is not None for p in group["params"]):
                    raise RuntimeError("cmve Adam(capturable=True): every parameter of a group needs a grad")
                dev_step = group.get("_dev_step")
                if dev_step is None:
                    dev_step = group["_dev_step"] = torch.zeros(1, dtype=torch.int64, device=ps[0].device)
            for p in ps:
                st = self.state[p]
                if not st:
                    st["step"] = dev_step if capturable else torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                if not capturable:
                    st["step"] += 1
                    steps.append(int(st["step"].item()))
            pa, sizes = _ptr_array(ps)
            ga, _ = _ptr_array([p.grad for p in ps])
            ma, _ = _ptr_array([self.state[p]["exp_avg"] for p in ps])
            va, _ = _ptr_array([self.state[p]["exp_avg_sq"] for p in ps])
            sa = (engine.C.c_int64 * len(ps))(*steps) if steps else None
            check(lib.cmve_adam_multi(_h(ps[0]), len(ps), pa, ga, ma, va, sizes, sa, float(group["lr"]), float(b1),
                                      float(b2), float(group["eps"]), float(group["weight_decay"]),
                                      _p(grad_scale), _p(dev_step)), "cmve_adam_multi")
            for p in ps:
                torch.autograd.graph.increment_version(p)  # the packed-weight caches key on _version
        return loss


# ---------------------------------------------------------------- train_emb
class GTTrainer:
    """The 'GT' training step of Dual_Encoding (model.py:984-1004) around the HIP heads.

    ``vid_encoder`` / ``text_encoder`` are the (PyTorch) encoders producing the mapping inputs, or
    None when the inputs are already encoder features (the C2 synthetic step pools frames with K2
    and feeds the pooled features).  Parameter order follows init_info (model.py:481-494)."""

    def __init__(self, vid_mapping, text_mapping, criterion, learning_rate=1e-4, grad_clip=2.0,
                 vid_encoder: Optional[nn.Module] = None, text_encoder: Optional[nn.Module] = None,
                 graph: bool = False):
        self.vid_encoding, self.text_encoding = vid_encoder, text_encoder
        self.vid_mapping, self.text_mapping = vid_mapping, text_mapping
        self.criterion = criterion
        self.grad_clip = grad_clip
        params = []
        for m in (vid_encoder, text_encoder, vid_mapping, text_mapping):
            if m is not None:
                params += list(m.parameters())
        self.params = params
        self.optimizer = Adam(self.params, lr=learning_rate, capturable=graph)
        self.Eiters = 0
        self.graph = graph
        self._graph = None
        self._warm = 0
        self._stream = None

    def train_start(self):
        for m in (self.vid_encoding, self.text_encoding, self.vid_mapping, self.text_mapping):
            if m is not None:
                m.train()

    def forward_emb(self, videos, captions):
        v = self.vid_encoding(videos) if self.vid_encoding is not None else videos
        c = self.text_encoding(captions) if self.text_encoding is not None else captions
        return self.vid_mapping(v), self.text_mapping(c)

    def forward_loss(self, cap_emb, vid_emb):
        return self.criterion(cap_emb, vid_emb)

    def train_emb(self, videos, captions, sync: bool = True):
        """Returns (batch size, loss value) like the reference; sync=False returns the loss as a
        device tensor instead of calling .item() (no host synchronisation inside the step).
        With graph=True the step is one hipGraph replay (see _graphed_step)."""
        if self.graph:
            bs, loss = self._graphed_step(videos, captions)
            return bs, (loss.item() if sync else loss)
        self.Eiters += 1
        vid_emb, cap_emb = self.forward_emb(videos, captions)
        self.optimizer.zero_grad()
        loss = self.forward_loss(cap_emb, vid_emb)
        loss_value = loss.item() if sync else loss.detach()
        loss.backward()
        coef = None
        if self.grad_clip > 0:  # clip_grad_norm_ fused into the Adam launch (same arithmetic, same grads)
            _, coef = clip_grad_norm_(self.params, self.grad_clip, _apply=False)
        self.optimizer.step(grad_scale=coef)
        return vid_emb.size(0), loss_value

    def _graphed_step(self, videos, captions):
        """The whole step (heads forward, loss, backward, clip, Adam: ~40 launches) captured once into a
        hipGraph and replayed: the first two calls run eagerly on the capture stream (creating its
        cmve handle and growing its scratch outside capture), the third captures and replays.  Every
        call is exactly one training step.  Inputs are copied into static buffers; the dropout stream
        position and the Adam step count live on the device, so replays advance them."""
        self.Eiters += 1
        cur = torch.cuda.current_stream(videos.device)
        if self._stream is None:
            self._stream = torch.cuda.Stream(videos.device)
        if self._graph is None and self._warm < 2:
            self._stream.wait_stream(cur)
            with torch.cuda.stream(self._stream):
                loss = self._eager_step(videos, captions)
            cur.wait_stream(self._stream)
            self._warm += 1
            return videos.size(0), loss
        if self._graph is None:
            self._static = (videos.clone(), captions.clone())
            self._graph = torch.cuda.CUDAGraph()
            self._stream.wait_stream(cur)
            with torch.cuda.graph(self._graph, stream=self._stream):
                self._static_loss = self._eager_step(*self._static)
        else:
            self._static[0].copy_(videos)
            self._static[1].copy_(captions)
        self._graph.replay()
        for p in self.params:
            torch.autograd.graph.increment_version(p)  # replays update the weights behind autograd's back
        return videos.size(0), self._static_loss

    def _eager_step(self, videos, captions):
        vid_emb, cap_emb = self.forward_emb(videos, captions)
        self.optimizer.zero_grad()
        loss = self.forward_loss(cap_emb, vid_emb)
        loss.backward()
        coef = None
        if self.grad_clip > 0:
            _, coef = clip_grad_norm_(self.params, self.grad_clip, _apply=False)
        self.optimizer.step(grad_scale=coef)
        return loss.detach()
