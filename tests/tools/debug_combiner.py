"""Stage-by-stage comparison of the GPU Combiner with the numpy oracle (debug aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root (tests/tools/..)
for p in (os.path.join(ROOT, "cross-modal-video-engine_amd"), ROOT, os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import numpy as np  # noqa
import torch  # noqa
import synth  # noqa
from cmve.multifusion import combiner as CC  # noqa
from cmve.linas.model import temporal_pool  # noqa

sd = synth.combiner_state()
sd64 = {k: v.astype(np.float64) for k, v in sd.items()}
m = CC.Combiner(640, 2560, 5120).cuda()
m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
m.eval()
b = 4
high, mid, text, _ = synth.combiner_inputs(b, 21)
d = 640
f, l = 8, 16


def cmp(name, gpu, ref):
    g = gpu.detach().cpu().numpy().astype(np.float64)
    print(f"{name:12s} max|diff| {np.abs(g - ref).max():.3e}  max|ref| {np.abs(ref).max():.3e}", flush=True)


dev = torch.device("cuda")
t_text = torch.from_numpy(text).to(dev)
t_mid = torch.from_numpy(mid).to(dev)
n = b * f
xt = t_mid.reshape(n, 640, 16).transpose(1, 2).reshape(n * 16, 640)
y = CC._linear(xt, m.m_remained.weight.view(640, -1), m.m_remained.bias, CC.ACT_RELU)
p_s_m = y.view(n, 16, -1).transpose(1, 2).reshape(b, f, l, -1)
X = mid.astype(np.float64).reshape(n, -1, 16)
Y = np.einsum("oc,ncp->nop", sd64["m_remained.weight"].reshape(640, 640), X) + sd64["m_remained.bias"][None, :, None]
ref_psm = np.maximum(Y, 0).reshape(b, f, l, -1)
cmp("p_s_m", p_s_m, ref_psm)
p_r_m = CC._linear(t_text, m.m_residual.weight, m.m_residual.bias, CC.ACT_RELU)
ref_prm = np.maximum(text @ sd64["m_residual.weight"].T + sd64["m_residual.bias"], 0)
cmp("p_r_m", p_r_m, ref_prm)
blk = m.self_attn_1
kv_in = p_s_m.reshape(l * f * b, d)
kv_ln = CC._layernorm(kv_in, blk.ln_1)
ref_kv = ref_psm.reshape(l * f * b, d)
mu = ref_kv.mean(-1, keepdims=True)
var = ((ref_kv - mu) ** 2).mean(-1, keepdims=True)
ref_kvln = (ref_kv - mu) / np.sqrt(var + 1e-5) * sd64["self_attn_1.ln_1.weight"] + sd64["self_attn_1.ln_1.bias"]
cmp("kv_ln", kv_ln, ref_kvln)
v3 = p_s_m.reshape(l * f, b, d)
v_mean = temporal_pool(v3.transpose(0, 1), "mean")
cmp("v_mean", v_mean, ref_psm.reshape(l * f, b, d).mean(0))
ref_mean = m.time_process(torch.from_numpy(high).to(dev))
cmp("ref_mean", ref_mean, high.astype(np.float64).mean(1))
out = m.combine_features((torch.from_numpy(high).to(dev), t_mid), t_text)
from oracle import combiner as OC  # noqa
cmp("final", out, OC.combine_features(sd, high, mid, text))
# ---- later stages ----
from cmve import engine  # noqa
from cmve._lib import lib, check  # noqa
W, Bi = blk.attn.in_proj_weight, blk.attn.in_proj_bias
q_ln = CC._layernorm(p_r_m, blk.ln_1)
q = CC._linear(q_ln, W[:d], Bi[:d])
kv = CC._linear(kv_ln, W[d:], Bi[d:])
mu = ref_prm.mean(-1, keepdims=True)
var = ((ref_prm - mu) ** 2).mean(-1, keepdims=True)
ref_qln = (ref_prm - mu) / np.sqrt(var + 1e-5) * sd64["self_attn_1.ln_1.weight"] + sd64["self_attn_1.ln_1.bias"]
Wi, bi = sd64["self_attn_1.attn.in_proj_weight"], sd64["self_attn_1.attn.in_proj_bias"]
ref_q = ref_qln @ Wi[:d].T + bi[:d]
ref_kvp = ref_kvln @ Wi[d:].T + bi[d:]
cmp("q", q, ref_q)
cmp("kv", kv, ref_kvp)
attn = torch.empty((b, d), dtype=torch.float32, device=dev)
check(lib.cmve_mha_1q(engine.handle(dev), engine._ptr(q), q.stride(0), engine._ptr(kv), kv.stride(0), d, b, l * f, 8,
                      80, engine._ptr(attn), attn.stride(0)))
kh = ref_kvp[:, :d].reshape(l * f, b, 8, 80)
vh = ref_kvp[:, d:].reshape(l * f, b, 8, 80)
qh = ref_q.reshape(b, 8, 80) * 80 ** -0.5
s = np.einsum("bhe,tbhe->bht", qh, kh)
s = np.exp(s - s.max(-1, keepdims=True)); p = s / s.sum(-1, keepdims=True)
ref_attn = np.einsum("bht,tbhe->bhe", p, vh).reshape(b, d)
cmp("attn", attn, ref_attn)
tp = CC._linear(t_text, m.text_projection_layer.weight, m.text_projection_layer.bias, CC.ACT_RELU)
cmp("tp", tp, np.maximum(text @ sd64["text_projection_layer.weight"].T + sd64["text_projection_layer.bias"], 0))
ip = CC._linear(ref_mean, m.image_projection_layer.weight, m.image_projection_layer.bias, CC.ACT_RELU)
ref_ip = np.maximum(high.astype(np.float64).mean(1) @ sd64["image_projection_layer.weight"].T + sd64["image_projection_layer.bias"], 0)
cmp("ip", ip, ref_ip)
raw = torch.cat((ip, tp), -1)
ref_raw = np.concatenate([ref_ip, np.maximum(text @ sd64["text_projection_layer.weight"].T + sd64["text_projection_layer.bias"], 0)], -1)
wcat, bcat = m._hidden_cat()
hid = CC._linear(raw, wcat, bcat, CC.ACT_RELU)
ref_comb = np.maximum(ref_raw @ sd64["combiner_layer.weight"].T + sd64["combiner_layer.bias"], 0)
ref_hid = np.maximum(ref_raw @ sd64["dynamic_scalar.0.weight"].T + sd64["dynamic_scalar.0.bias"], 0)
cmp("comb", hid[:, :5120], ref_comb)
cmp("dshid", hid[:, 5120:], ref_hid)
ds = CC._linear(hid[:, 5120:], m.dynamic_scalar[3].weight, m.dynamic_scalar[3].bias, CC.ACT_SIGMOID)
ref_ds = 1 / (1 + np.exp(-(ref_hid @ sd64["dynamic_scalar.3.weight"].T + sd64["dynamic_scalar.3.bias"])))
cmp("ds", ds, ref_ds)
yo = CC._linear(hid[:, :5120], m.output_layer.weight, m.output_layer.bias)
cmp("yo", yo, ref_comb @ sd64["output_layer.weight"].T + sd64["output_layer.bias"])
x = CC._linear(attn, blk.attn.out_proj.weight, blk.attn.out_proj.bias, resid=v_mean)
ref_x = ref_psm.reshape(l * f, b, d).mean(0) + ref_attn @ sd64["self_attn_1.attn.out_proj.weight"].T + sd64["self_attn_1.attn.out_proj.bias"]
cmp("x", x, ref_x)
ln2 = CC._layernorm(x, blk.ln_2)
mu = ref_x.mean(-1, keepdims=True); var = ((ref_x - mu) ** 2).mean(-1, keepdims=True)
ref_ln2 = (ref_x - mu) / np.sqrt(var + 1e-5) * sd64["self_attn_1.ln_2.weight"] + sd64["self_attn_1.ln_2.bias"]
cmp("ln2", ln2, ref_ln2)
h = CC._linear(ln2, blk.mlp.c_fc.weight, blk.mlp.c_fc.bias, CC.ACT_QUICKGELU)
ref_h = ref_ln2 @ sd64["self_attn_1.mlp.c_fc.weight"].T + sd64["self_attn_1.mlp.c_fc.bias"]
ref_h = ref_h / (1 + np.exp(-1.702 * ref_h))
cmp("h", h, ref_h)
based = CC._linear(h, blk.mlp.c_proj.weight, blk.mlp.c_proj.bias, resid=x)
ref_based = ref_x + ref_h @ sd64["self_attn_1.mlp.c_proj.weight"].T + sd64["self_attn_1.mlp.c_proj.bias"]
cmp("based", based, ref_based)
out2 = torch.empty_like(yo)
check(lib.cmve_fuse_combine(engine.handle(dev), engine._ptr(yo), engine._ptr(ds.contiguous()), engine._ptr(t_text),
                            engine._ptr(ref_mean), engine._ptr(based.contiguous()), b, d, 1e-12, engine._ptr(out2)))
ref_out = (ref_comb @ sd64["output_layer.weight"].T + sd64["output_layer.bias"]) + ref_ds * text + (1 - ref_ds) * high.astype(np.float64).mean(1) + np.maximum(ref_based, 0)
ref_out = ref_out / np.linalg.norm(ref_out, axis=-1, keepdims=True)
cmp("fused", out2, ref_out)
cmp("final_vs_dbg", out, out2.cpu().numpy().astype(np.float64))
