"""Combiner.combine_features / forward: oracle and GPU path vs the reference module's
outputs (tests/golden/combiner.npz), deterministic weights from synth.combiner_state()."""
import numpy as np
import pytest

import synth
from oracle import combiner as OC


@pytest.fixture(scope="module")
def state():
    return synth.combiner_state()


@pytest.mark.parametrize("b,seed", [(32, 21), (7, 22), (1, 23)])
def test_oracle_combine(golden, state, b, seed):
    g = golden("combiner")
    high, mid, text, _ = synth.combiner_inputs(b, seed)
    np.testing.assert_allclose(OC.combine_features(state, high, mid, text), g[f"pred_b{b}"], rtol=0, atol=2e-6)


def test_oracle_batch_mixing_and_logits(golden, state):
    g = golden("combiner")
    high, mid, text, tgt = synth.combiner_inputs(32, 21)
    alone = OC.combine_features(state, high[:7], mid[:7], text[:7])
    np.testing.assert_allclose(alone, g["pred_b32_first7_alone"], rtol=0, atol=2e-6)
    assert np.abs(alone - g["pred_b32"][:7]).max() > 1e-3  # the reference's batch dependence is real
    np.testing.assert_allclose(OC.forward_logits(state, high, mid, text, tgt), g["logits_b32"], rtol=0, atol=2e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("absorbed", [True, False])
def test_gpu_combiner(golden, state, absorbed):
    """Both attention paths against the reference module's outputs: K9b (K / V projections absorbed, keys read
    from the conv output, cmve_mha_absorbed) and the projected-K/V path (cmve_mha_1q)."""
    import torch
    from cmve.multifusion.combiner import Combiner
    g = golden("combiner")
    m = Combiner(640, 2560, 5120).cuda()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()})
    m.eval()
    m.absorbed = absorbed
    for b, seed in ((32, 21), (7, 22), (1, 23)):
        high, mid, text, tgt = synth.combiner_inputs(b, seed)
        pred = m.combine_features((torch.from_numpy(high).cuda(), torch.from_numpy(mid).cuda()),
                                  torch.from_numpy(text).cuda())
        np.testing.assert_allclose(pred.cpu().numpy(), g[f"pred_b{b}"], rtol=0, atol=1e-5)
        if b == 32:
            logits = m((torch.from_numpy(high).cuda(), torch.from_numpy(mid).cuda()), torch.from_numpy(text).cuda(),
                       (torch.from_numpy(tgt).cuda(),))
            np.testing.assert_allclose(logits.cpu().numpy(), g["logits_b32"], rtol=0, atol=1e-3)
    high, mid, text, _ = synth.combiner_inputs(32, 21)
    alone = m.combine_features((torch.from_numpy(high[:7]).cuda(), torch.from_numpy(mid[:7]).cuda()),
                               torch.from_numpy(text[:7]).cuda())
    np.testing.assert_allclose(alone.cpu().numpy(), g["pred_b32_first7_alone"], rtol=0, atol=1e-5)


@pytest.mark.gpu
def test_gpu_absorbed_attention_matches_projected(state):
    """K9b against the projected-K/V path on a C4-sized grouped batch (combine_batches, 8 batches of 32):
    the same function up to fp32 rounding (unit rows: 2e-6 absolute), and the absorbed weights follow a
    weight update (cache keyed on the parameters' versions)."""
    import torch
    from cmve.multifusion.combiner import Combiner
    m = Combiner(640, 2560, 5120).cuda()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()})
    m.eval()
    parts = [synth.combiner_inputs(32, 50 + i)[:3] for i in range(8)]
    high, mid, text = (torch.from_numpy(np.concatenate([p[j] for p in parts])).cuda() for j in range(3))
    a = m.combine_batches((high, mid), text)
    m.absorbed = False
    p = m.combine_batches((high, mid), text)
    assert (a - p).abs().max().item() < 2e-6
    with torch.no_grad():
        m.self_attn_1.attn.in_proj_weight.mul_(1.5)
        m.self_attn_1.ln_1.weight.add_(0.25)
    p2 = m.combine_batches((high, mid), text)
    m.absorbed = True
    a2 = m.combine_batches((high, mid), text)
    assert (a2 - p2).abs().max().item() < 2e-6 and (a2 - a).abs().max().item() > 1e-4


@pytest.mark.gpu
def test_gpu_combine_batches_equals_batch_loop(state):
    """combine_batches (all full 32-row batches in one pass, per-batch attention layout rebuilt) is
    bit-identical to validate.py's loop of combine_features over consecutive batches of 32, the
    last partial batch (7 rows) included; and it still mixes rows within each batch only."""
    import torch
    from cmve.multifusion.combiner import Combiner
    m = Combiner(640, 2560, 5120).cuda()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()})
    m.eval()
    parts = [synth.combiner_inputs(32, 31 + i)[:3] for i in range(3)] + [synth.combiner_inputs(7, 40)[:3]]
    high, mid, text = (torch.from_numpy(np.concatenate([p[j] for p in parts])).cuda() for j in range(3))
    loop = torch.cat([m.combine_features((high[i:i + 32], mid[i:i + 32]), text[i:i + 32])
                      for i in range(0, high.shape[0], 32)])
    fused = m.combine_batches((high, mid), text, batch_size=32)
    assert torch.equal(loop, fused)


@pytest.mark.gpu
def test_gpu_fused_transpose_and_layernorm_packing():
    """cmve_pack_tblocks / cmve_layernorm_pack write the same split-bf16 planes cmve_pack_rows
    (raw rows) makes of the fp32 transpose / LayerNorm, bit for bit, padding rows / columns zero;
    cmve_transpose_blocks equals the torch transpose."""
    import torch
    from cmve import engine
    from cmve.multifusion.combiner import _layernorm
    rng = np.random.default_rng(5)
    x = torch.from_numpy(rng.standard_normal((37, 16, 640)).astype(np.float32)).cuda()
    ref_t = x.reshape(37, 640, 16).transpose(1, 2).reshape(37 * 16, 640).contiguous()
    op = engine.PackedOperand.from_blocks_transposed(x, 640, 16)
    rs = engine.RowSet(ref_t, with_lo=True, with_f16=False, raw_rows=True)
    assert op.n == rs.n and op.n_pad >= rs.n_pad
    assert torch.equal(op.hi[:rs.n_pad], rs.hi) and torch.equal(op.lo[:rs.n_pad], rs.lo)
    assert not op.hi[rs.n_pad:].any()
    y = torch.from_numpy(rng.standard_normal((37 * 16, 640)).astype(np.float32)).cuda()
    assert torch.equal(engine.transpose_blocks(y, 16, 640),
                       y.view(37, 16, 640).transpose(1, 2).reshape(37 * 640, 16))
    ln = torch.nn.LayerNorm(200).cuda()
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
    z = torch.from_numpy(rng.standard_normal((333, 200)).astype(np.float32)).cuda()
    pk = engine.PackedOperand.layernorm(z, ln.weight, ln.bias, ln.eps)
    rz = engine.RowSet(_layernorm(z, ln), with_lo=True, with_f16=False, raw_rows=True)
    assert torch.equal(pk.hi, rz.hi) and torch.equal(pk.lo, rz.lo)


@pytest.mark.gpu
@pytest.mark.parametrize("d,strided", [(640, False), (200, True), (201, False), (1024, False), (1500, False)])
def test_gpu_layernorm_paths(d, strided):
    """cmve_layernorm (float4 rows when d % 4 == 0 and the rows are aligned, else the scalar rows)
    against an fp64 LayerNorm, and cmve_layernorm_pack equal to packing its output, bit for bit."""
    import torch
    from cmve import engine
    from cmve.multifusion.combiner import _layernorm
    rng = np.random.default_rng(d)
    ln = torch.nn.LayerNorm(d).cuda()
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
    base = torch.from_numpy((3 * rng.standard_normal((517, d + 8)) + 1).astype(np.float32)).cuda()
    z = base[:, :d].contiguous()
    y = _layernorm(z, ln)
    if strided:  # rows at a 4-byte offset with ldx = d + 8: the scalar-row kernel on the same values
        from cmve._lib import lib
        zs = base[:, 1:1 + d]
        zs.copy_(z)
        ys = torch.empty_like(z)
        assert lib.cmve_layernorm(engine.handle(z.device), engine._ptr(zs), zs.stride(0), zs.shape[0], d,
                                  engine._ptr(ln.weight.detach()), engine._ptr(ln.bias.detach()), float(ln.eps),
                                  engine._ptr(ys), ys.stride(0)) == 0
        assert (ys - y).abs().max().item() < 1e-6
    if d % 4 == 0 and d <= 1024:  # aligned input, misaligned output: the same (float4-row) sums, bit for bit
        from cmve._lib import lib
        ybig = torch.empty((z.shape[0], d + 3), dtype=torch.float32, device=z.device)
        yo = ybig[:, 1:1 + d]
        assert lib.cmve_layernorm(engine.handle(z.device), engine._ptr(z), z.stride(0), z.shape[0], d,
                                  engine._ptr(ln.weight.detach()), engine._ptr(ln.bias.detach()), float(ln.eps),
                                  engine._ptr(yo), yo.stride(0)) == 0
        assert torch.equal(yo, y)
    z64 = z.double()
    ref = torch.nn.functional.layer_norm(z64, (d,), ln.weight.double(), ln.bias.double(), ln.eps)
    assert (y.double() - ref).abs().max().item() < 2e-6
    if d <= 1024:
        pk = engine.PackedOperand.layernorm(z, ln.weight, ln.bias, ln.eps)
        rz = engine.RowSet(y, with_lo=True, with_f16=False, raw_rows=True)
        assert torch.equal(pk.hi, rz.hi) and torch.equal(pk.lo, rz.lo)


@pytest.mark.gpu
@pytest.mark.parametrize("R,C", [(5, 7), (16, 12), (12, 16)])
def test_gpu_transpose_blocks_shapes(R, C):
    """Block transposes on the scalar (C or R not a multiple of 4) and float4 forms, against torch."""
    import torch
    from cmve import engine
    y = torch.randn(9 * R * C, generator=torch.Generator().manual_seed(R * C)).cuda()
    ref = y.view(9, R, C).transpose(1, 2).reshape(9 * C, R)
    assert torch.equal(engine.transpose_blocks(y, R, C), ref)
    op = engine.PackedOperand.from_blocks_transposed(y.view(9, R, C), R, C)
    rs = engine.RowSet(ref.contiguous(), with_lo=True, with_f16=False, raw_rows=True)
    assert torch.equal(op.hi[:rs.n_pad], rs.hi) and torch.equal(op.lo[:rs.n_pad], rs.lo)


@pytest.mark.gpu
@pytest.mark.parametrize("d,f,gs,B", [(640, 8, 32, 64), (512, 4, 5, 15), (640, 2, 7, 7)])
def test_gpu_mha_absorbed_against_fp64(d, f, gs, B):
    """cmve_mha_absorbed (K9b) through the C ABI against an fp64 torch restatement of its contract: key t of
    query qb = g*gs + bb is run R % L of conv block g*gs*f + R / L (R = t*gs + bb) of y [B*f*16, C = d];
    z_h = sum_t softmax_t(u_h . n_t) n_t with n_t the un-affined LayerNorm of the key (eps 1e-5), in the kernel's
    element order (e = p*cpr + c' <-> original c'*16 + p), and v.mean(0) in the original order."""
    import torch
    from cmve import engine
    from cmve._lib import lib, check
    H, npix = 8, 16
    cpr, L = d // npix, d // (d // npix)
    T = f * L
    gen = torch.Generator().manual_seed(d + f + gs)
    y = torch.relu(torch.randn(B * f * npix, d, generator=gen, dtype=torch.float64))
    u = torch.randn(B, H * d, generator=gen, dtype=torch.float64) * 0.05
    yc, uc = y.float().cuda(), u.float().cuda()
    z = torch.empty(B, H * d, device="cuda")
    vm = torch.empty(B, d, device="cuda")
    check(lib.cmve_mha_absorbed(engine.handle(yc.device), engine._ptr(yc), yc.stride(0), d, npix, f, gs, B, H, d,
                                engine._ptr(uc), uc.stride(0), 1e-5, engine._ptr(z), z.stride(0), engine._ptr(vm),
                                vm.stride(0)), "cmve_mha_absorbed")
    yd, ud = yc.double().cpu(), uc.double().cpu()
    p_idx, c_idx = torch.meshgrid(torch.arange(npix), torch.arange(cpr), indexing="ij")
    perm = (c_idx * npix + p_idx).reshape(-1)  # kernel element e -> original element
    zr = torch.empty(B, H, d, dtype=torch.float64)
    vr = torch.empty(B, d, dtype=torch.float64)
    for qb in range(B):
        g, bb = divmod(qb, gs)
        keys = []
        for t in range(T):
            R = t * gs + bb
            bf, run = g * gs * f + R // L, R % L
            blk = yd[bf * npix:(bf + 1) * npix, run * cpr:(run + 1) * cpr]  # [p, c']
            keys.append(blk.reshape(-1))  # kernel order e = p*cpr + c'
        X = torch.stack(keys)  # [T, d] kernel order
        n = (X - X.mean(1, keepdim=True)) / torch.sqrt(X.var(1, unbiased=False, keepdim=True) + 1e-5)
        s = n @ ud[qb].view(H, d).T  # [T, H]
        p = torch.softmax(s, 0)
        zr[qb] = p.T @ n
        orig = torch.empty_like(X)
        orig[:, perm] = X
        vr[qb] = orig.mean(0)
    assert (z.double().cpu().view(B, H, d) - zr).abs().max().item() < 2e-5
    assert (vm.double().cpu() - vr).abs().max().item() < 2e-6
