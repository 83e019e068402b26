"""MultiFusion Combiner training step on libcmve.so.

``CombinerTrainer.train_step`` is the loop body of MultiFusion/src/combiner_train.py:341-381::

    optimizer.zero_grad()
    logits = combiner(ref, text_features, target)      # Combiner.forward in train mode (dropout 0.5)
    loss = CrossEntropyLoss()(logits, arange(B))       # K7 InfoNCE, row half, scale = logit_scale
    scaler.scale(loss).backward(); scaler.step(optimizer); scaler.update()

``combiner_train_forward`` is Combiner.forward / combine_features (MultiFusion/src/combiner.py:121-180)
as a chain of autograd functions, each a HIP kernel forward and backward:

    Linear / 1x1 conv / in-projection   cmve_gemm_f32(_ex) (K11's exact-fp32 MFMA GEMM, cmve.linas.train.linear)
    ReLU / Sigmoid / QuickGELU          cmve_act_fwd / _bwd (K16)
    LayerNorm ln_1 / ln_2               cmve_layernorm_train_fwd / _bwd (K16)
    attention (1 query per batch row)   cmve_mha_1q / cmve_mha_1q_bwd (K8 / K16)
    raw-reshape transposes              cmve_transpose_blocks (both directions)
    time_process mean                   cmve_temporal_pool / cmve_pool_mean_bwd
    output fusion                       cmve_combine_train_fwd / _bwd (K16)
    F.normalize                         cmve_l2norm_rows / cmve_l2norm_bwd
    dropout                             cmve_dropout / cmve_mask_scale (K11: same distribution, NOT torch's stream)

Precision: the reference runs the step under torch.cuda.amp.autocast (fp16 GEMMs) with a GradScaler;
this step computes in fp32 throughout (exact-fp32 GEMMs), so there is nothing for a loss scaler to
protect: ``scaler`` is accepted for interface parity and only its skip-on-inf rule is kept (a step
whose gradients are not finite is skipped, as GradScaler.step does).
"""
from __future__ import annotations

import torch

from .. import engine
from .._lib import lib, check, ACT_RELU_K, ACT_SIGMOID_K, ACT_QUICKGELU_K
from ..linas.train import Adam, linear, dropout
from .loss import InfoNCE

_p = engine._ptr


def _h(t):
    return engine.handle(t.device)


def _f32(t):
    t = t.detach()
    t = t if t.dtype == torch.float32 else t.float()
    return t if t.is_contiguous() else t.contiguous()


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kind):
        xs = _f32(x)
        y = torch.empty_like(xs)
        check(lib.cmve_act_fwd(_h(xs), _p(xs), xs.numel(), kind, _p(y)), "cmve_act_fwd")
        ctx.save_for_backward(xs)
        ctx.kind = kind
        return y

    @staticmethod
    def backward(ctx, dy):
        (xs,) = ctx.saved_tensors
        dy = _f32(dy)
        dx = torch.empty_like(xs)
        check(lib.cmve_act_bwd(_h(xs), _p(xs), _p(dy), xs.numel(), ctx.kind, _p(dx)), "cmve_act_bwd")
        return dx, None


def relu(x):
    return _ActFn.apply(x, ACT_RELU_K)


def sigmoid(x):
    return _ActFn.apply(x, ACT_SIGMOID_K)


def quick_gelu(x):
    return _ActFn.apply(x, ACT_QUICKGELU_K)


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        xs = _f32(x)
        n, d = xs.shape
        y = torch.empty_like(xs)
        mean = torch.empty(n, dtype=torch.float32, device=xs.device)
        rstd = torch.empty(n, dtype=torch.float32, device=xs.device)
        g, b = _f32(gamma), _f32(beta)
        check(lib.cmve_layernorm_train_fwd(_h(xs), _p(xs), d, n, d, _p(g), _p(b), float(eps), _p(y), d, _p(mean),
                                           _p(rstd)), "cmve_layernorm_train_fwd")
        ctx.save_for_backward(xs, g, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, g, mean, rstd = ctx.saved_tensors
        dy = _f32(dy)
        n, d = xs.shape
        dx = torch.empty_like(xs)
        dg = torch.empty(d, dtype=torch.float32, device=xs.device)
        db = torch.empty(d, dtype=torch.float32, device=xs.device)
        check(lib.cmve_layernorm_bwd(_h(xs), _p(xs), d, _p(dy), d, n, d, _p(g), _p(mean), _p(rstd), _p(dx), d, _p(dg),
                                     _p(db)), "cmve_layernorm_bwd")
        return dx, dg, db, None


def layer_norm(x, ln):
    return _LayerNormFn.apply(x, ln.weight, ln.bias, ln.eps)


class _MHA1QFn(torch.autograd.Function):
    """out[b] = attention of query b over keys / values at rows t*B + b of kv (K | V columns)."""

    @staticmethod
    def forward(ctx, q, kv, B, T, H):
        qs, kvs = _f32(q), _f32(kv)
        d = qs.shape[1]
        out = torch.empty((B, d), dtype=torch.float32, device=qs.device)
        check(lib.cmve_mha_1q(_h(qs), _p(qs), qs.stride(0), _p(kvs), kvs.stride(0), d, B, T, H, d // H, _p(out),
                              out.stride(0)), "cmve_mha_1q")
        ctx.save_for_backward(qs, kvs)
        ctx.cfg = (B, T, H)
        return out

    @staticmethod
    def backward(ctx, dout):
        qs, kvs = ctx.saved_tensors
        B, T, H = ctx.cfg
        d = qs.shape[1]
        dout = _f32(dout)
        dq = torch.empty_like(qs)
        dkv = torch.empty_like(kvs)
        check(lib.cmve_mha_1q_bwd(_h(qs), _p(qs), qs.stride(0), _p(kvs), kvs.stride(0), d, B, T, H, d // H, _p(dout),
                                  dout.stride(0), _p(dq), dq.stride(0), _p(dkv), dkv.stride(0)), "cmve_mha_1q_bwd")
        return dq, dkv, None, None, None


class _BlockTransposeFn(torch.autograd.Function):
    """[nb][R][C] -> [nb * C, R] (cmve_transpose_blocks); the backward is the inverse transpose."""

    @staticmethod
    def forward(ctx, x, R, C):
        ctx.cfg = (R, C)
        return engine.transpose_blocks(x, R, C)

    @staticmethod
    def backward(ctx, dy):
        R, C = ctx.cfg
        return engine.transpose_blocks(_f32(dy), C, R).view(-1), None, None


class _MeanFn(torch.autograd.Function):
    """time_process: x [B, T, F] -> mean over T (K2 MEAN_ALL)."""

    @staticmethod
    def forward(ctx, x):
        from ..linas.model import temporal_pool
        ctx.shape = tuple(x.shape)
        return temporal_pool(_f32(x), "mean")

    @staticmethod
    def backward(ctx, dy):
        B, T, F = ctx.shape
        dy = _f32(dy)
        dx = torch.empty((B, T, F), dtype=torch.float32, device=dy.device)
        check(lib.cmve_pool_mean_bwd(_h(dy), _p(dy), B, T, F, _p(dx)), "cmve_pool_mean_bwd")
        return dx


class _CombineFn(torch.autograd.Function):
    """((y + ds*text) + (1-ds)*ref) + based, ds [B, 1] (combiner.py:178-179)."""

    @staticmethod
    def forward(ctx, y, ds, text, ref, based):
        ys, dss, ts, rs, bs = (_f32(t) for t in (y, ds, text, ref, based))
        B, d = ys.shape
        out = torch.empty_like(ys)
        check(lib.cmve_combine_train_fwd(_h(ys), _p(ys), _p(dss), _p(ts), _p(rs), _p(bs), B, d, _p(out)),
              "cmve_combine_train_fwd")
        ctx.save_for_backward(dss, ts, rs)
        return out

    @staticmethod
    def backward(ctx, g):
        dss, ts, rs = ctx.saved_tensors
        g = _f32(g)
        B, d = g.shape
        dt = torch.empty_like(ts) if ctx.needs_input_grad[2] else None
        dr = torch.empty_like(rs) if ctx.needs_input_grad[3] else None
        dds = torch.empty((B, 1), dtype=torch.float32, device=g.device)
        check(lib.cmve_combine_train_bwd(_h(g), _p(g), _p(dss), _p(ts), _p(rs), B, d, _p(dt), _p(dr), _p(dds)),
              "cmve_combine_train_bwd")
        return g, dds, dt, dr, g


class _NormalizeFn(torch.autograd.Function):
    """F.normalize(x, dim=-1) (eps 1e-12; the backward is the exact one for rows with ||x|| > eps)."""

    @staticmethod
    def forward(ctx, x):
        from .validate import normalize
        xs = _f32(x)
        ctx.save_for_backward(xs)
        return normalize(xs)

    @staticmethod
    def backward(ctx, dy):
        (xs,) = ctx.saved_tensors
        dy = _f32(dy)
        dx = torch.empty_like(xs)
        check(lib.cmve_l2norm_bwd(_h(xs), _p(xs), xs.stride(0), _p(dy), dy.stride(0), xs.shape[0], xs.shape[1],
                                  _p(dx), dx.stride(0)), "cmve_l2norm_bwd")
        return dx


def _drop(x, module, training):
    return dropout(x, module.p, training) if training else x


def combine_features_train(combiner, image_features, text_features):
    """Combiner.combine_features (combiner.py:146-180) with autograd, module in train mode."""
    tr = combiner.training
    ref_high, ref_mid = image_features
    ref_high = _f32(ref_high)
    ref_mid = _f32(ref_mid)
    text = text_features if text_features.requires_grad else _f32(text_features)
    b, f, l, d = ref_mid.shape
    C = ref_mid[0, 0].numel() // 16
    # 1x1 conv over ref_mid.reshape(b*f, C, 4, 4): rows (n, pixel) of the [C, 16] blocks
    x_rows = _BlockTransposeFn.apply(ref_mid.reshape(-1), C, 16)                    # [b*f*16, C]
    conv = combiner.m_remained
    y_rows = linear(x_rows, conv.weight.view(conv.weight.shape[0], -1), conv.bias)  # [b*f*16, C_out]
    y_nchw = _BlockTransposeFn.apply(y_rows.reshape(-1), 16, conv.weight.shape[0])  # [(n, o), 16] = NCHW
    p_s_m = _drop(relu(y_nchw), combiner.dropout7, tr).reshape(b, f, l, -1)
    p_r_m = _drop(relu(linear(text, combiner.m_residual.weight, combiner.m_residual.bias)), combiner.dropout6, tr)
    # ResidualAttentionBlock(q = p_r_m [1, b, d], k = v = p_s_m.reshape(l*f, b, d))  (combiner.py:38-43,164-165)
    blk = combiner.self_attn_1
    kv_in = p_s_m.reshape(l * f * b, d)                                             # row t*b + bb
    W, Bi = blk.attn.in_proj_weight, blk.attn.in_proj_bias
    q = linear(layer_norm(p_r_m, blk.ln_1), W[:d], Bi[:d])
    kv = linear(layer_norm(kv_in, blk.ln_1), W[d:], Bi[d:])                          # [l*f*b, 2d]: K | V
    attn = _MHA1QFn.apply(q, kv, b, l * f, blk.attn.num_heads)
    attn = linear(attn, blk.attn.out_proj.weight, blk.attn.out_proj.bias)
    v_mean = _MeanFn.apply(kv_in.reshape(l * f, b, d).transpose(0, 1).contiguous())  # v.mean(dim=0)
    x = v_mean + attn
    hmid = quick_gelu(linear(layer_norm(x, blk.ln_2), blk.mlp.c_fc.weight, blk.mlp.c_fc.bias))
    x = x + linear(hmid, blk.mlp.c_proj.weight, blk.mlp.c_proj.bias)
    based = _drop(relu(x), combiner.dropout4, tr)
    # projections, combiner and dynamic scalar (combiner.py:168-175)
    ref_mean = _MeanFn.apply(ref_high)
    tp = _drop(relu(linear(text, combiner.text_projection_layer.weight, combiner.text_projection_layer.bias)),
               combiner.dropout1, tr)
    ip = _drop(relu(linear(ref_mean, combiner.image_projection_layer.weight, combiner.image_projection_layer.bias)),
               combiner.dropout2, tr)
    raw = torch.cat((ip, tp), -1)
    combined = _drop(relu(linear(raw, combiner.combiner_layer.weight, combiner.combiner_layer.bias)),
                     combiner.dropout3, tr)
    dsm = combiner.dynamic_scalar
    hds = _drop(relu(linear(raw, dsm[0].weight, dsm[0].bias)), dsm[2], tr)
    ds = sigmoid(linear(hds, dsm[3].weight, dsm[3].bias))                            # [b, 1]
    yo = linear(combined, combiner.output_layer.weight, combiner.output_layer.bias)
    out = _CombineFn.apply(yo, ds, text, ref_mean, based)
    return _NormalizeFn.apply(out)


def combiner_train_forward(combiner, image_features, text_features, target_features):
    """Combiner.forward (combiner.py:121-138) with autograd: the predicted features and the
    normalised time-pooled target (the logits are formed inside the CE, scale logit_scale)."""
    pred = combine_features_train(combiner, image_features, text_features)
    tgt = _NormalizeFn.apply(_MeanFn.apply(_f32(target_features[0])))
    return pred, tgt


class CombinerTrainer:
    """The training loop body of combiner_train.py:341-381 on the cmve kernels; Adam over
    combiner.parameters() (combiner_train.py:316)."""

    def __init__(self, combiner, lr: float = 2e-6, scaler=None):
        self.combiner = combiner
        self.optimizer = Adam(list(combiner.parameters()), lr=lr)
        self.criterion = InfoNCE(scale=float(combiner.logit_scale), direction="row")
        self.scaler = scaler
        self.skipped = 0

    def train_step(self, reference, text_features, target, sync: bool = True):
        """reference = (high [B, f, d], middle [B, f, l, d]), target = (high, middle); returns the loss."""
        self.combiner.train()
        self.optimizer.zero_grad()
        pred, tgt = combiner_train_forward(self.combiner, reference, text_features, target)
        loss = self.criterion(pred, tgt)          # CE(100 * pred @ tgt^T, arange(B))
        loss.backward()
        if self.scaler is not None:  # GradScaler.step: skip the update when a gradient is not finite
            finite = torch.stack([torch.isfinite(p.grad).all() for p in self.combiner.parameters()
                                  if p.grad is not None]).all()
            if not bool(finite):
                self.skipped += 1
                return loss.item() if sync else loss.detach()
        self.optimizer.step()
        return loss.item() if sync else loss.detach()
