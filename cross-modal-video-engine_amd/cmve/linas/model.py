"""Mirror of the LINAS projection heads / pools (``LINAS-engine/model.py``) on libcmve.so.

  l2norm(X)                               model.py:35-40   (row L2, no epsilon)
  MFC(fc_layers, dropout, ...)            model.py:51-116  (eval forward: fused GEMM epilogue, K3)
  Latent_mapping(mapping_layers, ...)     model.py:362-381 (MFC + BN + l2norm)
  temporal pools                          model.py:152-166 (gru mean / masked max / max_pool1d)
  Video_multilevel_encoding(opt)          model.py:119-188 (eval forward: frozen biGRU / Conv2d in
                                          PyTorch-ROCm, every pool on K2)
Modules keep the reference's parameter names, so reference checkpoints load with
``load_state_dict`` (slot layout model.py:387-404).  Inference (eval) runs on the HIP kernels;
training mode (batch-statistics BN, dropout, autograd backward) runs on the K11 functions of
``cmve.linas.train``.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from .. import engine
from .._lib import lib, check, SIM_BF16X3, POOL_MEAN_VALID, POOL_MEAN_ALL, POOL_MAX_MASKED_ZERO, POOL_MAX_ALL


def l2norm(X: torch.Tensor) -> torch.Tensor:
    """X / ||X|| per row, no epsilon (zero row -> NaN), on the GPU."""
    X = X.detach()
    if not X.is_cuda:
        raise RuntimeError("cmve.linas.model.l2norm expects a device tensor")
    dt = X.dtype if X.dtype in (torch.float32, torch.float64) else torch.float32
    x = X.to(dt).contiguous()
    out = torch.empty_like(x)
    if x.shape[0]:
        check(lib.cmve_l2norm_rows(engine.handle(x.device), engine._ptr(x), engine._dtype_code(x), x.stride(0),
                                   engine._ptr(out), engine._dtype_code(out), out.stride(0), x.shape[0], x.shape[1],
                                   0.0), "cmve_l2norm_rows")
    return out


def temporal_pool(x: torch.Tensor, mode: str, lengths=None) -> torch.Tensor:
    """x [B, T, F] fp32 device -> [B, F].  mode: 'mean_valid' (first lengths[b] steps),
    'mean' (all T), 'masked_max' (max_t x*mask, masked steps = 0), 'max' (all T)."""
    codes = {"mean_valid": POOL_MEAN_VALID, "mean": POOL_MEAN_ALL, "masked_max": POOL_MAX_MASKED_ZERO,
             "max": POOL_MAX_ALL}
    m = codes[mode]
    x = x.detach().to(torch.float32)
    if x.stride(2) != 1:
        x = x.contiguous()
    B, T, F = x.shape
    out = torch.empty((B, F), dtype=torch.float32, device=x.device)
    lens = None
    if m in (POOL_MEAN_VALID, POOL_MAX_MASKED_ZERO):
        lens = torch.as_tensor(np.asarray(lengths, np.int32) if not torch.is_tensor(lengths) else lengths,
                               dtype=torch.int32).to(x.device)
    if B:
        check(lib.cmve_temporal_pool(engine.handle(x.device), engine._ptr(x), x.stride(0), x.stride(1), B, T, F,
                                     engine._ptr(lens), m, engine._ptr(out), out.stride(0)), "cmve_temporal_pool")
    return out


class _PackedWeight:
    """A linear layer's weight [F_out, K] packed (split-bf16, raw) once, on first use."""

    def __init__(self):
        self.key = None
        self.rows = None

    def get(self, w: torch.Tensor):
        key = (w.data_ptr(), w._version, tuple(w.shape), w.device)
        if self.key != key:
            self.rows = engine.RowSet(w.detach().float(), with_lo=True, with_f16=False, raw_rows=True,
                                      device=w.device)
            self.key = key
        return self.rows


def linear_fused(x: torch.Tensor, weight: torch.Tensor, bias=None, relu=False, resid=None, bn=None,
                 packed: _PackedWeight = None, out: torch.Tensor = None) -> torch.Tensor:
    """out = BN(resid + act(x W^T + b)) on the split-bf16 MFMA kernel (K3); `out` (fp32 [n, F_out], rows
    contiguous, any row stride) receives it in place when given."""
    x = x.detach().float().contiguous()
    xr = engine.RowSet(x, with_lo=True, with_f16=False, raw_rows=True, device=x.device)
    wr = (packed or _PackedWeight()).get(weight)
    if out is None:
        out = torch.empty((x.shape[0], weight.shape[0]), dtype=torch.float32, device=x.device)
    elif (out.dtype != torch.float32 or tuple(out.shape) != (x.shape[0], weight.shape[0]) or out.stride(1) != 1
          or out.device != x.device):
        raise ValueError(f"linear_fused: out must be fp32 [{x.shape[0]}, {weight.shape[0]}] on {x.device}")
    scale = shift = None
    if bn is not None:
        scale, shift = bn
    b = bias.detach().float().contiguous() if bias is not None else None
    r = resid.contiguous() if resid is not None else None
    check(lib.cmve_linear(engine.handle(x.device), engine.C.byref(xr.desc), engine.C.byref(wr.desc), SIM_BF16X3,
                          engine._ptr(b), engine._ptr(scale), engine._ptr(shift), engine._ptr(r),
                          r.stride(0) if r is not None else 0, 1 if relu else 0, engine._ptr(out), out.stride(0)),
          "cmve_linear")
    return out


def bn_eval_affine(bn: nn.BatchNorm1d):
    """BatchNorm1d eval as a per-column affine (scale, shift), computed in fp64."""
    w = bn.weight.detach().double() if bn.weight is not None else torch.ones_like(bn.running_var, dtype=torch.float64)
    b = bn.bias.detach().double() if bn.bias is not None else torch.zeros_like(bn.running_var, dtype=torch.float64)
    inv = 1.0 / torch.sqrt(bn.running_var.detach().double() + bn.eps)
    scale = w * inv
    shift = b - bn.running_mean.detach().double() * scale
    return scale.float().contiguous(), shift.float().contiguous()


def _xavier_init_fc(fc: nn.Linear):
    r = np.sqrt(6.) / np.sqrt(fc.in_features + fc.out_features)  # model.py:43-49
    fc.weight.data.uniform_(-r, r)
    fc.bias.data.fill_(0)


class MFC(nn.Module):
    """Multi fully-connected layers (model.py:51-116) -- same submodule names / state dict."""

    def __init__(self, fc_layers, dropout, have_dp=True, have_bn=False, have_last_bn=False):
        super().__init__()
        self.n_fc = len(fc_layers)
        if self.n_fc > 1:
            for k in range(1, min(self.n_fc, 5)):
                setattr(self, f"fc{k}", nn.Linear(fc_layers[k - 1], fc_layers[k]))
            self.relu = nn.ReLU()
            self.have_dp = have_dp
            if have_dp:
                self.dropout = nn.Dropout(p=dropout)
            self.have_bn = have_bn
            self.have_last_bn = have_last_bn
            if have_bn and have_last_bn:
                self.bn_1 = nn.BatchNorm1d(fc_layers[-1])
            for k in range(1, min(self.n_fc, 5)):
                _xavier_init_fc(getattr(self, f"fc{k}"))
        self._packed = {}

    def forward(self, inputs):
        if self.n_fc <= 1:
            return inputs
        if self.training:  # batch-statistics BN, dropout, autograd backward (cmve.linas.train, K11)
            from .train import mfc_train_forward
            return mfc_train_forward(self, inputs)
        n_lin = min(self.n_fc, 5) - 1
        bn = bn_eval_affine(self.bn_1) if (self.have_bn and self.have_last_bn) else None
        feats = None
        x = inputs
        for k in range(1, n_lin + 1):
            fc = getattr(self, f"fc{k}")
            pk = self._packed.setdefault(k, _PackedWeight())
            last = k == n_lin
            bnk = bn if last else None
            if k == 1:
                feats = linear_fused(x, fc.weight, fc.bias, bn=bnk, packed=pk)
            else:  # features = features + relu(fc_k(features))   (model.py:104-109)
                feats = linear_fused(feats, fc.weight, fc.bias, relu=True, resid=feats, bn=bnk, packed=pk)
        return feats  # dropout is identity in eval


class Latent_mapping(nn.Module):
    """model.py:362-381: MFC(have_bn=True, have_last_bn=True) then l2norm."""

    def __init__(self, mapping_layers, dropout, l2norm=True):
        super().__init__()
        self.l2norm = l2norm
        self.mapping = MFC(mapping_layers, dropout, have_bn=True, have_last_bn=True)

    def forward(self, features):
        latent = self.mapping(features)
        if self.l2norm:
            if self.training:
                from .train import l2norm_train
                latent = l2norm_train(latent)
            else:
                latent = globals()["l2norm"](latent)
        return latent


def video_level_features(gru_init_out, videos_mask, lengths, videos_origin, convs, gru_pool="mean",
                         concate="full"):
    """The pooling skeleton of Video_multilevel_encoding.forward (model.py:143-176) around the frozen
    biGRU / Conv2d backbones: pools on the HIP kernels, conv stays PyTorch-ROCm (frozen backbone)."""
    if gru_pool == "mean":
        gru_out = temporal_pool(gru_init_out, "mean_valid", lengths)
    else:
        gru_out = temporal_pool(gru_init_out, "masked_max", lengths)
    masked = gru_init_out * videos_mask.unsqueeze(2)
    con_in = masked.unsqueeze(1)
    con_out = [torch.relu(conv(con_in)).squeeze(3) for conv in convs]       # [B, C, T']
    con_out = [temporal_pool(c.transpose(1, 2).contiguous(), "max") for c in con_out]
    con_out = torch.cat(con_out, 1)
    if concate == "full":
        return torch.cat((gru_out, con_out, videos_origin), 1)
    return torch.cat((gru_out, con_out), 1)


class Video_multilevel_encoding(nn.Module):
    """model.py:119-188, eval forward.  Same submodule names (``rnn``, ``convs1``) and state-dict
    keys as the reference, so its checkpoint slots load unchanged; the biGRU and the Conv2d bank
    are the frozen backbones (PyTorch-ROCm), the temporal pools run on K2 (video_level_features).

    As in the reference the GRU runs over the zero-padded batch (no packing, model.py:150), and
    the conv max-pool spans the batch's padded width, so an embedding depends on the batch it is
    encoded in (the collate of encode_vid fixes that batch)."""

    def __init__(self, opt):
        super().__init__()
        self.rnn_output_size = opt.visual_rnn_size * 2
        self.dropout = nn.Dropout(p=opt.dropout)
        self.concate = opt.concate
        self.gru_pool = opt.gru_pool
        self.tag_vocab_size = getattr(opt, "tag_vocab_size", None)
        self.loss_fun = getattr(opt, "loss_fun", "mrl")
        self.rnn = nn.GRU(opt.visual_feat_dim, opt.visual_rnn_size, batch_first=True, bidirectional=True)
        self.convs1 = nn.ModuleList([
            nn.Conv2d(1, opt.visual_kernel_num, (w, self.rnn_output_size), padding=(w - 1, 0))
            for w in opt.visual_kernel_sizes])

    def forward(self, videos):
        if self.training:
            raise NotImplementedError("cmve Video_multilevel_encoding is the frozen gallery-side backbone: "
                                      "call .eval()")
        vids, videos_origin, lengths, videos_mask = videos
        with torch.no_grad():
            gru_init_out, _ = self.rnn(vids)
            return video_level_features(gru_init_out, videos_mask, lengths, videos_origin, self.convs1,
                                        gru_pool=self.gru_pool, concate=self.concate)

    def load_state_dict(self, state_dict, strict=True):
        """model.py:178-188: keep only this module's keys (a full model's state dict loads)."""
        own = self.state_dict()
        return super().load_state_dict({k: v for k, v in state_dict.items() if k in own}, strict=strict)
