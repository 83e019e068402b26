"""CPU oracle (numpy, fp64) of MultiFusion Combiner.combine_features / forward (eval).

TEST INFRASTRUCTURE ONLY (see oracle/retrieval.py).  Restates MultiFusion/src/combiner.py:19-43
(ResidualAttentionBlock) and :121-180, including the raw reshapes that mix the batch
(:159, :164-165).  Pinned to tests/golden/combiner.npz, produced by the reference module itself.
"""
from __future__ import annotations

import numpy as np


def _ln(x, g, b, eps=1e-5):
    m = x.mean(-1, keepdims=True)
    v = ((x - m) ** 2).mean(-1, keepdims=True)
    return (x - m) / np.sqrt(v + eps) * g + b


def _relu(x):
    return np.maximum(x, 0.0)


def combine_features(sd, high, mid, text, n_head=8):
    sd = {k: np.asarray(v, np.float64) for k, v in sd.items()}
    high = np.asarray(high, np.float64)
    mid = np.asarray(mid, np.float64)
    text = np.asarray(text, np.float64)
    b, f, l, d = mid.shape
    X = mid.reshape(b * f, -1, 16)                                          # (b*f, C, 4*4)  combiner.py:159
    W = sd["m_remained.weight"].reshape(sd["m_remained.weight"].shape[0], -1)
    Y = np.einsum("oc,ncp->nop", W, X) + sd["m_remained.bias"][None, :, None]
    p_s_m = _relu(Y).reshape(b, f, l, -1)
    p_r_m = _relu(text @ sd["m_residual.weight"].T + sd["m_residual.bias"])
    q = p_r_m.reshape(-1, b, d)                                            # [1, b, d]
    kv = p_s_m.reshape(l * f, b, d)                                        # raw reshape: mixes the batch
    g1, b1 = sd["self_attn_1.ln_1.weight"], sd["self_attn_1.ln_1.bias"]
    Wi, bi = sd["self_attn_1.attn.in_proj_weight"], sd["self_attn_1.attn.in_proj_bias"]
    qp = _ln(q, g1, b1) @ Wi[:d].T + bi[:d]
    kp = _ln(kv, g1, b1) @ Wi[d:2 * d].T + bi[d:2 * d]
    vp = _ln(kv, g1, b1) @ Wi[2 * d:].T + bi[2 * d:]
    dh = d // n_head
    qh = qp.reshape(1, b, n_head, dh) * dh ** -0.5
    kh = kp.reshape(l * f, b, n_head, dh)
    vh = vp.reshape(l * f, b, n_head, dh)
    s = np.einsum("qbhe,tbhe->bht", qh, kh)
    s = np.exp(s - s.max(-1, keepdims=True))
    p = s / s.sum(-1, keepdims=True)
    o = np.einsum("bht,tbhe->bhe", p, vh).reshape(b, d)
    attn = o @ sd["self_attn_1.attn.out_proj.weight"].T + sd["self_attn_1.attn.out_proj.bias"]
    x = kv.mean(axis=0) + attn                                             # v.mean(dim=0) + attn
    h = _ln(x, sd["self_attn_1.ln_2.weight"], sd["self_attn_1.ln_2.bias"]) @ sd["self_attn_1.mlp.c_fc.weight"].T \
        + sd["self_attn_1.mlp.c_fc.bias"]
    h = h * (1.0 / (1.0 + np.exp(-1.702 * h)))                             # QuickGELU
    x = x + h @ sd["self_attn_1.mlp.c_proj.weight"].T + sd["self_attn_1.mlp.c_proj.bias"]
    based = _relu(x)
    ref = high.mean(axis=1)                                                # time_process
    tp = _relu(text @ sd["text_projection_layer.weight"].T + sd["text_projection_layer.bias"])
    ip = _relu(ref @ sd["image_projection_layer.weight"].T + sd["image_projection_layer.bias"])
    raw = np.concatenate([ip, tp], -1)
    comb = _relu(raw @ sd["combiner_layer.weight"].T + sd["combiner_layer.bias"])
    hid = _relu(raw @ sd["dynamic_scalar.0.weight"].T + sd["dynamic_scalar.0.bias"])
    ds = 1.0 / (1.0 + np.exp(-(hid @ sd["dynamic_scalar.3.weight"].T + sd["dynamic_scalar.3.bias"])))
    out = comb @ sd["output_layer.weight"].T + sd["output_layer.bias"] + ds * text + (1 - ds) * ref + based
    return out / np.maximum(np.linalg.norm(out, axis=-1, keepdims=True), 1e-12)


def forward_logits(sd, high, mid, text, target_high, scale=100.0):
    pred = combine_features(sd, high, mid, text)
    t = np.asarray(target_high, np.float64).mean(axis=1)
    t = t / np.maximum(np.linalg.norm(t, axis=-1, keepdims=True), 1e-12)
    return scale * pred @ t.T
