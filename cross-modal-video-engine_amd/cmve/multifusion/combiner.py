"""Mirror of MultiFusion's ``Combiner`` (MultiFusion/src/combiner.py:81-180) on libcmve.so (eval).

Same constructor, submodule names and state-dict keys as the reference, so a reference
checkpoint ``{'Combiner': state_dict}`` (MultiFusion/src/inference.py:213-223) loads directly.
``combine_features`` / ``forward`` / ``time_process`` run on the HIP kernels:
  conv1x1 on the raw (b*f, d, 4, 4) reshape, projections, in/out projections, MLP, combiner
  and dynamic-scalar layers -> cmve_linear (split-bf16 MFMA, fused bias/act/residual epilogue);
  LayerNorm -> cmve_layernorm; the 1-query x 128-key attention over the batch-mixing
  p_s_m.reshape(l*f, b, d) (combiner.py:164-165) -> cmve_mha_1q; v.mean(0) and time_process ->
  cmve_temporal_pool; the residual combine + F.normalize -> cmve_fuse_combine.
PyTorch only re-lays memory (reshape / transpose / cat), exactly as the reference's reshapes.
The batch-composition dependence of the reference is therefore reproduced.
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn as nn

from .. import engine
from .._lib import lib, check, SIM_BF16X3
from ..linas.model import linear_fused, temporal_pool, _PackedWeight

ACT_NONE, ACT_RELU, ACT_QUICKGELU, ACT_SIGMOID = 0, 1, 2, 3


def _linear(x, w, b, act=ACT_NONE, resid=None, packed=None):
    if isinstance(x, engine.PackedOperand):  # operand already packed by a fused kernel
        xr = x
    else:
        x = x.detach().float().contiguous()
        xr = engine.RowSet(x, with_lo=True, with_f16=False, raw_rows=True, device=x.device)
    wr = packed.get(w) if packed is not None else _PackedWeight().get(w)
    out = torch.empty((xr.n, w.shape[0]), dtype=torch.float32, device=xr.device)
    bb = b.detach().float().contiguous() if b is not None else None
    r = resid.contiguous() if resid is not None else None
    check(lib.cmve_linear(engine.handle(xr.device), engine.C.byref(xr.desc), engine.C.byref(wr.desc), SIM_BF16X3,
                          engine._ptr(bb), None, None, engine._ptr(r), r.stride(0) if r is not None else 0, act,
                          engine._ptr(out), out.stride(0)), "cmve_linear")
    return out


def _layernorm(x, ln: nn.LayerNorm):
    x = x.contiguous().float()
    y = torch.empty_like(x)
    n, d = x.shape
    check(lib.cmve_layernorm(engine.handle(x.device), engine._ptr(x), x.stride(0), n, d,
                             engine._ptr(ln.weight.detach().float().contiguous()),
                             engine._ptr(ln.bias.detach().float().contiguous()), float(ln.eps), engine._ptr(y),
                             y.stride(0)), "cmve_layernorm")
    return y


class QuickGELU(nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(1.702 * x)


class ResidualAttentionBlock(nn.Module):
    """combiner.py:19-43 -- parameters only; the forward is fused in Combiner.combine_features."""

    def __init__(self, d_model: int, n_head: int):
        super().__init__()
        self.attn = nn.MultiheadAttention(d_model, n_head)
        self.ln_1 = nn.LayerNorm(d_model)
        self.mlp = nn.Sequential(OrderedDict([("c_fc", nn.Linear(d_model, d_model * 4)), ("gelu", QuickGELU()),
                                              ("c_proj", nn.Linear(d_model * 4, d_model))]))
        self.ln_2 = nn.LayerNorm(d_model)


class Combiner(nn.Module):
    def __init__(self, clip_feature_dim: int, projection_dim: int, hidden_dim: int):
        super().__init__()
        self.text_projection_layer = nn.Linear(clip_feature_dim, projection_dim)
        self.image_projection_layer = nn.Linear(clip_feature_dim, projection_dim)
        self.dropout1 = nn.Dropout(0.5)
        self.dropout2 = nn.Dropout(0.5)
        self.combiner_layer = nn.Linear(projection_dim * 2, hidden_dim)
        self.output_layer = nn.Linear(hidden_dim, clip_feature_dim)
        self.dropout3 = nn.Dropout(0.5)
        self.dynamic_scalar = nn.Sequential(nn.Linear(projection_dim * 2, hidden_dim), nn.ReLU(), nn.Dropout(0.5),
                                            nn.Linear(hidden_dim, 1), nn.Sigmoid())
        self.logit_scale = 100
        self.m_remained = nn.Conv2d(clip_feature_dim, clip_feature_dim, (1, 1))
        self.m_residual = nn.Linear(clip_feature_dim, clip_feature_dim)
        self.nhead = 8
        self.self_attn_1 = ResidualAttentionBlock(clip_feature_dim, self.nhead)
        self.dropout4 = nn.Dropout(0.5)
        self.dropout6 = nn.Dropout(0.5)
        self.dropout7 = nn.Dropout(0.5)
        self._pk = {}
        # K9b absorbed attention (fusion.hip); False = the projected-K/V path (cmve_mha_1q), kept for A/B and tests
        self.absorbed = True
        self._cat_key = None
        self._cat_w = self._cat_b = None

    def _p(self, name):
        return self._pk.setdefault(name, _PackedWeight())

    def _hidden_cat(self):
        """combiner_layer and dynamic_scalar[0] read the same input: one GEMM with both weights."""
        a, b = self.combiner_layer, self.dynamic_scalar[0]
        key = (a.weight.data_ptr(), a.weight._version, b.weight.data_ptr(), b.weight._version)
        if self._cat_key != key:
            self._cat_w = torch.cat([a.weight.detach(), b.weight.detach()], 0).float().contiguous()
            self._cat_b = torch.cat([a.bias.detach(), b.bias.detach()], 0).float().contiguous()
            self._cat_key = key
        return self._cat_w, self._cat_b

    def _absorbed(self, npix: int):
        """The attention's K / V in-projections absorbed (fusion.hip K9b, combiner.py:38-40): per head h
        (dh = d / H, gamma / beta = ln_1's affine, perm = the kernel's element order within a key run,
        e = p * (d / npix) + c' <-> original c' * npix + p):
          M[h d + e, :] = gamma_j / sqrt(dh) * (W_k,h^T W_q,h)[j, :],  c[h d + e] = gamma_j / sqrt(dh) * (W_k,h^T b_q,h)_j
          N[:, h d + e] = (W_o,h W_v,h)[:, j] * gamma_j,               bN = W_o (W_v beta + b_v) + b_o
        with j = perm[e]: scores u_h . n_t equal q'_h . K_t,h / sqrt(dh) up to terms constant over the keys, and
        z @ N^T + bN equals out_proj(concat_h sum_t p_t V_t,h).  Formed in fp64, stored fp32, cached per weight
        version."""
        blk = self.self_attn_1
        W, Bi = blk.attn.in_proj_weight, blk.attn.in_proj_bias
        Wo, bo = blk.attn.out_proj.weight, blk.attn.out_proj.bias
        g, be = blk.ln_1.weight, blk.ln_1.bias
        key = tuple((t.data_ptr(), t._version) for t in (W, Bi, Wo, bo, g, be)) + (npix,)
        if getattr(self, "_abs_key", None) != key:
            d, H = W.shape[1], self.nhead
            dh, cpr = d // H, d // npix
            Wd, bd = W.detach().double(), Bi.detach().double()
            Wq, Wk, Wv = Wd[:d], Wd[d:2 * d], Wd[2 * d:]
            bq, bv = bd[:d], bd[2 * d:]
            Wod, bod = Wo.detach().double(), bo.detach().double()
            gd, bed = g.detach().double(), be.detach().double()
            p, c = torch.meshgrid(torch.arange(npix), torch.arange(cpr), indexing="ij")
            perm = (c * npix + p).reshape(-1).to(W.device)
            sc = 1.0 / (dh ** 0.5)
            Ms, cs, Ns = [], [], []
            for h in range(H):
                sl = slice(h * dh, (h + 1) * dh)
                Ms.append(((Wk[sl].t() @ Wq[sl]) * (gd * sc)[:, None])[perm])
                cs.append(((Wk[sl].t() @ bq[sl]) * gd * sc)[perm])
                Ns.append(((Wod[:, sl] @ Wv[sl]) * gd[None, :])[:, perm])
            self._abs_M = torch.cat(Ms, 0).float().contiguous()
            self._abs_c = torch.cat(cs, 0).float().contiguous()
            self._abs_N = torch.cat(Ns, 1).float().contiguous()
            self._abs_bN = (Wod @ (Wv @ bed + bv) + bod).float().contiguous()
            self._abs_key = key
        return self._abs_M, self._abs_c, self._abs_N, self._abs_bN

    def time_process(self, fea):
        """combiner.py:140-143: mean over the frame axis."""
        return temporal_pool(fea, "mean")

    @torch.no_grad()
    def combine_features(self, image_features, text_features):
        """combiner.py:146-180 on one batch (the raw reshapes mix the whole batch)."""
        return self._combine(image_features, text_features, None)

    @torch.no_grad()
    def combine_batches(self, image_features, text_features, batch_size: int = 32):
        """Equal to concatenating combine_features over consecutive batches of ``batch_size`` rows
        (validate.py:207-208's loop; the last partial batch is its own batch), bit for bit -- but the
        full batches run as ONE pass: every GEMM / LayerNorm / pool is row-wise, and the attention's
        batch-mixing key layout (combiner.py:164-165) is rebuilt per batch (keys of query (g, bb) at
        rows t * B + g * batch_size + bb), so the GEMMs see M = all rows instead of one batch."""
        ref_high, ref_mid = image_features
        n = ref_mid.shape[0]
        full = (n // batch_size) * batch_size
        outs = []
        if full:
            outs.append(self._combine((ref_high[:full], ref_mid[:full]), text_features[:full], batch_size))
        if full < n:
            outs.append(self._combine((ref_high[full:], ref_mid[full:]), text_features[full:], None))
        return torch.cat(outs) if len(outs) > 1 else outs[0]

    def _combine(self, image_features, text_features, group):
        if self.training:
            raise NotImplementedError("cmve Combiner: eval-mode forward only (training is SURVEY 8f 'next')")
        ref_high, ref_mid = image_features
        ref_high = ref_high.float()
        ref_mid = ref_mid.float()
        text = text_features.float().contiguous()
        b, f, l, d = ref_mid.size()
        gs = b if group is None else int(group)
        if b % gs:
            raise ValueError("combine_batches: rows must be a multiple of the batch size")
        G = b // gs
        n = b * f
        # conv1x1 over the raw reshape (b*f, -1, 4, 4) (combiner.py:159): channel c = elements c*16 .. c*16+15,
        # so the GEMM rows are the 16 columns of each [C, 16] block -- packed straight from ref_mid
        C = ref_mid[0, 0].numel() // 16
        xt = engine.PackedOperand.from_blocks_transposed(ref_mid, C, 16)
        wc = self.m_remained.weight.view(self.m_remained.weight.shape[0], -1)
        y = _linear(xt, wc, self.m_remained.bias, ACT_RELU, packed=self._p("m_remained"))
        p_r_m = _linear(text, self.m_residual.weight, self.m_residual.bias, ACT_RELU, packed=self._p("m_residual"))
        # ResidualAttentionBlock(q = p_r_m [1,b,d], k = v = p_s_m.reshape(l*f, b, d))  combiner.py:38-43,164-165,
        # p_s_m = relu(conv).reshape(b, f, l, -1): the key/value rows, row t*b + bb == [t, bb] of the raw
        # reshape(l*f, b, d); with G batches of gs rows each batch's raw reshape is taken separately and
        # interleaved, row t*b + g*gs + bb -- written in that order straight from the conv output
        blk = self.self_attn_1
        q_ln = _layernorm(p_r_m, blk.ln_1)
        if self.absorbed and d % 16 == 0 and (d, self.nhead) in ((640, 8), (512, 8)):
            # K9b: K / V projections absorbed (see _absorbed); the keys are read straight from the conv output
            M, cu, N, bN = self._absorbed(16)
            u = _linear(q_ln, M, cu, packed=self._p("abs_m"))                # [b, H d]
            z = torch.empty((b, self.nhead * d), dtype=torch.float32, device=text.device)
            v_mean = torch.empty((b, d), dtype=torch.float32, device=text.device)
            check(lib.cmve_mha_absorbed(engine.handle(text.device), engine._ptr(y), y.stride(0), y.shape[1], 16, f, gs,
                                        b, self.nhead, d, engine._ptr(u), u.stride(0), float(blk.ln_1.eps),
                                        engine._ptr(z), z.stride(0), engine._ptr(v_mean), v_mean.stride(0)),
                  "cmve_mha_absorbed")
            x = _linear(z, N, bN, resid=v_mean, packed=self._p("abs_n"))
        else:
            kv_in = engine.transpose_blocks_kv(y, 16, y.shape[1], d, l * f, gs, b)
            kv_ln = engine.PackedOperand.layernorm(kv_in, blk.ln_1.weight, blk.ln_1.bias, blk.ln_1.eps)
            W, Bi = blk.attn.in_proj_weight, blk.attn.in_proj_bias
            q = _linear(q_ln, W[:d], Bi[:d], packed=self._p("in_q"))
            kv = _linear(kv_ln, W[d:], Bi[d:], packed=self._p("in_kv"))          # [l*f*b, 2d]: K | V
            attn = torch.empty((b, d), dtype=torch.float32, device=text.device)
            check(lib.cmve_mha_1q(engine.handle(text.device), engine._ptr(q), q.stride(0), engine._ptr(kv),
                                  kv.stride(0), d, b, l * f, self.nhead, d // self.nhead, engine._ptr(attn),
                                  attn.stride(0)), "cmve_mha_1q")
            v3 = kv_in.view(l * f, b, d)
            v_mean = temporal_pool(v3.transpose(0, 1), "mean")                    # v.mean(dim=0), strided view
            x = _linear(attn, blk.attn.out_proj.weight, blk.attn.out_proj.bias, resid=v_mean,
                        packed=self._p("out_proj"))
        h = _linear(_layernorm(x, blk.ln_2), blk.mlp.c_fc.weight, blk.mlp.c_fc.bias, ACT_QUICKGELU,
                    packed=self._p("c_fc"))
        based = _linear(h, blk.mlp.c_proj.weight, blk.mlp.c_proj.bias, resid=x, packed=self._p("c_proj"))
        # projections, combiner and dynamic scalar (combiner.py:168-175)
        ref_mean = self.time_process(ref_high)
        tp = _linear(text, self.text_projection_layer.weight, self.text_projection_layer.bias, ACT_RELU,
                     packed=self._p("tp"))
        ip = _linear(ref_mean, self.image_projection_layer.weight, self.image_projection_layer.bias, ACT_RELU,
                     packed=self._p("ip"))
        raw = torch.cat((ip, tp), -1)
        wcat, bcat = self._hidden_cat()
        hid = _linear(raw, wcat, bcat, ACT_RELU, packed=self._p("hidden_cat"))
        hd = self.combiner_layer.weight.shape[0]
        combined = hid[:, :hd]
        ds = _linear(hid[:, hd:], self.dynamic_scalar[3].weight, self.dynamic_scalar[3].bias, ACT_SIGMOID,
                     packed=self._p("ds3"))
        yo = _linear(combined, self.output_layer.weight, self.output_layer.bias, packed=self._p("out"))
        out = torch.empty_like(yo)
        check(lib.cmve_fuse_combine(engine.handle(text.device), engine._ptr(yo), engine._ptr(ds.contiguous()),
                                    engine._ptr(text), engine._ptr(ref_mean), engine._ptr(based.contiguous()), b, d,
                                    1e-12, engine._ptr(out)), "cmve_fuse_combine")
        return out

    @torch.no_grad()
    def forward(self, image_features, text_features, target_features):
        """combiner.py:121-138: logits = 100 * pred @ normalize(time_process(target[0])).T"""
        pred = self.combine_features(image_features, text_features)
        tgt = self.time_process(target_features[0].float())
        qp = engine.RowSet(pred, with_lo=True, with_f16=False, raw_rows=True, device=pred.device)
        tg = engine.RowSet(tgt, eps=1e-12, with_lo=True, with_f16=False, device=pred.device)
        return engine.sim_store(qp, tg, alpha=float(self.logit_scale), mode=SIM_BF16X3)
