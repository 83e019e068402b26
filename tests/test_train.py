"""Training-step row: the LINAS heads trained on the K11 / K3 / K6 kernels.

Golden vectors: tests/golden/train_step.npz and train_bn_l2.npz, from the reference's own
Latent_mapping (training mode), TripletLoss, clip_grad_norm_ and torch.optim.Adam driven as
train_emb 'GT' does (tests/golden/make_golden_train.py).
Tolerances: the reference runs fp32; the oracle fp64; the HIP path fp32 with fp64 statistics and
a split-bf16 forward GEMM (~1e-6 relative).  Gradients agree to ~1e-7 absolute.  One parameter is
special: the bias of a Linear feeding BatchNorm directly (vid fc1.bias) has an exactly-zero true
gradient, so every implementation's is rounding noise, and Adam turns noise of any size into steps
of ~lr.  That bias (and the running mean it shifts) is checked to within lr per step.
"""
import numpy as np
import pytest
import torch

from oracle import train as OT

LR, CLIP, STEPS = 1e-3, 2.0, 3
VID_N, TXT_N = 1, 2                  # linear layers per head (= make_golden_train layers)
NOISE_PARAMS = {"vid.mapping.fc1.bias"}


def _P(g, prefix, n_lin):
    d = {}
    for k in range(1, n_lin + 1):
        d[f"fc{k}.weight"] = g[f"{prefix}mapping.fc{k}.weight"]
        d[f"fc{k}.bias"] = g[f"{prefix}mapping.fc{k}.bias"]
    d["bn.weight"] = g[f"{prefix}mapping.bn_1.weight"]
    d["bn.bias"] = g[f"{prefix}mapping.bn_1.bias"]
    return d


def _run(g, prefix):
    return [g[f"{prefix}mapping.bn_1.running_mean"], g[f"{prefix}mapping.bn_1.running_var"]]


def _sd(g, prefix):
    return {k[len(prefix):]: torch.from_numpy(np.asarray(g[k])) for k in g.files if k.startswith(prefix)}


def test_oracle_matches_reference_golden(golden):
    g = golden("train_step")
    st = OT.GTStep(_P(g, "init_vid.", VID_N), VID_N, _run(g, "init_vid."), _P(g, "init_txt.", TXT_N), TXT_N,
                   _run(g, "init_txt."), LR, CLIP)
    for t in range(STEPS):
        loss, total, flat, vid, cap = st.step(g[f"step{t}_videos"], g[f"step{t}_captions"])
        np.testing.assert_allclose(loss, g[f"step{t}_loss"], rtol=1e-6)
        np.testing.assert_allclose(total, g[f"step{t}_total_norm"], rtol=1e-6)
        np.testing.assert_allclose(vid, g[f"step{t}_vid_emb"], atol=1e-6)
        np.testing.assert_allclose(cap, g[f"step{t}_cap_emb"], atol=1e-6)
        for i, f in enumerate(flat):
            np.testing.assert_allclose(f, g[f"step{t}_grad{i}"], rtol=1e-5, atol=1e-7)
    for hi, pre in ((0, "final_vid."), (1, "final_txt.")):
        fin = _P(g, pre, (VID_N, TXT_N)[hi])
        for k, v in fin.items():
            name = ("vid." if hi == 0 else "txt.") + "mapping." + k.replace("bn.", "bn_1.")
            atol = 1.1 * LR * STEPS if name in NOISE_PARAMS else 1e-6
            np.testing.assert_allclose(st.heads[hi][0][k], v, rtol=0, atol=atol, err_msg=name)
    np.testing.assert_allclose(st.heads[1][2][0], g["final_txt.mapping.bn_1.running_mean"], atol=1e-6)
    np.testing.assert_allclose(st.heads[1][2][1], g["final_txt.mapping.bn_1.running_var"], rtol=1e-6)
    np.testing.assert_allclose(st.heads[0][2][0], g["final_vid.mapping.bn_1.running_mean"], atol=0.1 * 1.1 * LR * STEPS)

    b = golden("train_bn_l2")
    P = {"fc1.weight": b["init.mapping.fc1.weight"], "fc1.bias": b["init.mapping.fc1.bias"],
         "bn.weight": b["init.mapping.bn_1.weight"], "bn.bias": b["init.mapping.bn_1.bias"]}
    y, tape = OT.mapping_forward(b["x"], P, 1)
    dx, gr = OT.mapping_backward(b["G"].astype(np.float64), P, 1, tape)
    np.testing.assert_allclose(y, b["y"], atol=1e-6)
    np.testing.assert_allclose(dx, b["dx"], atol=1e-6)
    for k in ("fc1.weight", "bn.weight", "bn.bias"):
        np.testing.assert_allclose(gr[k], b["grad.mapping." + k.replace("bn.", "bn_1.")], rtol=1e-5, atol=1e-6)


# ------------------------------------------------------------------ GPU
def _heads(g, prefix_v, prefix_t):
    from cmve.linas.model import Latent_mapping
    vm = Latent_mapping([96, 64], 0.0).cuda()
    tm = Latent_mapping([80, 64, 64], 0.0).cuda()
    vm.load_state_dict(_sd(g, prefix_v))
    tm.load_state_dict(_sd(g, prefix_t))
    return vm, tm


@pytest.mark.gpu
def test_latent_mapping_train_forward_backward_matches_reference(golden):
    from cmve.linas.model import Latent_mapping
    b = golden("train_bn_l2")
    lm = Latent_mapping([48, 40], 0.0).cuda()
    lm.load_state_dict(_sd(b, "init."))
    lm.train()
    x = torch.from_numpy(b["x"]).cuda().requires_grad_(True)
    y = lm(x)
    (y * torch.from_numpy(b["G"]).cuda()).sum().backward()
    np.testing.assert_allclose(y.detach().cpu().numpy(), b["y"], atol=2e-6)
    np.testing.assert_allclose(x.grad.cpu().numpy(), b["dx"], atol=2e-6)
    for k, p in lm.named_parameters():
        if k == "mapping.fc1.bias":  # exactly-zero true gradient (feeds BN): both sides are noise
            assert np.abs(p.grad.cpu().numpy()).max() < 1e-5
            continue
        np.testing.assert_allclose(p.grad.cpu().numpy(), b[f"grad.{k}"], rtol=1e-4, atol=2e-6, err_msg=k)
    after = _sd(b, "after.")
    for k, v in lm.state_dict().items():
        if "running" in k or "num_batches" in k:
            np.testing.assert_allclose(v.cpu().numpy(), after[k].numpy(), rtol=1e-5, atol=1e-6, err_msg=k)


@pytest.mark.gpu
def test_gt_train_step_matches_reference(golden):
    from cmve.linas.loss import TripletLoss
    from cmve.linas.train import GTTrainer
    g = golden("train_step")
    vm, tm = _heads(g, "init_vid.", "init_txt.")
    tr = GTTrainer(vm, tm, TripletLoss(margin=0.2, measure='cosine', max_violation=True, cost_style='sum',
                                       direction='all'), learning_rate=LR, grad_clip=CLIP)
    tr.train_start()
    for t in range(STEPS):
        bs, loss = tr.train_emb(torch.from_numpy(g[f"step{t}_videos"]).cuda(),
                                torch.from_numpy(g[f"step{t}_captions"]).cuda())
        assert bs == 32
        np.testing.assert_allclose(loss, g[f"step{t}_loss"], rtol=2e-6)
    names = list(g["param_names"])
    for i, p in enumerate(tr.params):
        fin = g[("final_vid." if names[i].startswith("vid.") else "final_txt.") + names[i][4:]]
        atol = 1.1 * LR * STEPS if names[i] in NOISE_PARAMS else 2e-6
        np.testing.assert_allclose(p.detach().cpu().numpy(), fin, rtol=0, atol=atol, err_msg=names[i])
        st = tr.optimizer.state[p]
        if names[i] not in NOISE_PARAMS:
            np.testing.assert_allclose(st["exp_avg"].cpu().numpy(), g[f"adam{i}_exp_avg"], rtol=1e-4, atol=1e-8)
            np.testing.assert_allclose(st["exp_avg_sq"].cpu().numpy(), g[f"adam{i}_exp_avg_sq"], rtol=1e-4,
                                       atol=1e-12)
        assert float(st["step"]) == STEPS
    for m, pre in ((vm, "final_vid."), (tm, "final_txt.")):
        sd = m.state_dict()
        assert int(sd["mapping.bn_1.num_batches_tracked"]) == STEPS
        np.testing.assert_allclose(sd["mapping.bn_1.running_var"].cpu().numpy(), g[pre + "mapping.bn_1.running_var"],
                                   rtol=1e-5)
    np.testing.assert_allclose(tm.state_dict()["mapping.bn_1.running_mean"].cpu().numpy(),
                               g["final_txt.mapping.bn_1.running_mean"], atol=2e-6)
    # eval after training sees the updated weights (packed-weight caches keyed on _version)
    from oracle.heads import latent_mapping_eval
    tm.eval()
    x = torch.from_numpy(g["step0_captions"]).cuda()
    want = latent_mapping_eval(g["step0_captions"], {k: v.cpu().numpy() for k, v in tm.state_dict().items()},
                               [80, 64, 64])
    np.testing.assert_allclose(tm(x).cpu().numpy(), want, atol=1e-5)  # eval GEMM: split-bf16 K3


@pytest.mark.gpu
@pytest.mark.parametrize("momentum,affine,n", [(0.1, True, 128), (None, True, 7), (0.3, False, 2)])
def test_batchnorm_train_matches_torch(momentum, affine, n):
    from cmve.linas.train import batch_norm_train
    torch.manual_seed(0)
    d = 200
    ref = torch.nn.BatchNorm1d(d, momentum=momentum, affine=affine).cuda().double()
    mine = torch.nn.BatchNorm1d(d, momentum=momentum, affine=affine).cuda()
    if affine:
        with torch.no_grad():
            ref.weight.uniform_(0.5, 1.5)
            ref.bias.normal_()
            mine.weight.copy_(ref.weight)
            mine.bias.copy_(ref.bias)
    for step in range(2):
        x = (torch.randn(n, d, device="cuda") * 3 + 1).requires_grad_(True)
        xr = x.detach().double().requires_grad_(True)
        G = torch.randn(n, d, device="cuda")
        y = batch_norm_train(x, mine)
        yr = ref(xr)
        (y * G).sum().backward()
        (yr * G.double()).sum().backward()
        torch.testing.assert_close(y.double(), yr, rtol=1e-5, atol=2e-5)
        torch.testing.assert_close(x.grad.double(), xr.grad, rtol=1e-4, atol=2e-5)
        torch.testing.assert_close(mine.running_mean.double(), ref.running_mean, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(mine.running_var.double(), ref.running_var, rtol=1e-5, atol=1e-6)
        assert int(mine.num_batches_tracked) == int(ref.num_batches_tracked)
        if affine:
            torch.testing.assert_close(mine.weight.grad.double(), ref.weight.grad, rtol=1e-4, atol=1e-4)
            torch.testing.assert_close(mine.bias.grad.double(), ref.bias.grad, rtol=1e-5, atol=1e-5)
            mine.weight.grad = mine.bias.grad = ref.weight.grad = ref.bias.grad = None
    from cmve._lib import CmveError
    with pytest.raises(CmveError, match="more than 1 value"):
        batch_norm_train(torch.randn(1, d, device="cuda"), mine)


@pytest.mark.gpu
@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_adam_and_clip_match_torch(wd):
    from cmve.linas.train import Adam, clip_grad_norm_
    torch.manual_seed(1)
    shapes = [(300, 77), (77,), (1,), (1024, 5)] + [(i + 1, 3) for i in range(27)]  # > 24: two launches
    ps = [torch.randn(s, device="cuda", requires_grad=True) for s in shapes]
    qs = [p.detach().clone().requires_grad_(True) for p in ps]
    mine, ref = Adam(ps, lr=3e-3, weight_decay=wd), torch.optim.Adam(qs, lr=3e-3, weight_decay=wd)
    for step in range(5):
        for p, q in zip(ps, qs):
            gr = torch.randn_like(p) * (0.5 if step % 2 else 4.0)
            p.grad, q.grad = gr.clone(), gr.clone()
        tn = clip_grad_norm_(ps, 1.5)
        tr = torch.nn.utils.clip_grad_norm_(qs, 1.5)
        torch.testing.assert_close(tn, tr, rtol=1e-6, atol=0)
        for p, q in zip(ps, qs):
            torch.testing.assert_close(p.grad, q.grad, rtol=2e-6, atol=1e-8)
        mine.step()
        ref.step()
        for p, q in zip(ps, qs):
            torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-6, atol=1e-7)
    sr = ref.state[qs[0]]
    sm = mine.state[ps[0]]
    torch.testing.assert_close(sm["exp_avg_sq"], sr["exp_avg_sq"], rtol=1e-5, atol=1e-10)
    assert float(sm["step"]) == float(sr["step"]) == 5


@pytest.mark.gpu
def test_dropout_mask_statistics_and_backward():
    from cmve.linas import train as T
    T.manual_seed(123)
    x = torch.randn(512, 1000, device="cuda", requires_grad=True)
    p = 0.2
    y = T.dropout(x, p)
    keep = (y != 0)
    frac = keep.float().mean().item()
    assert abs(frac - (1 - p)) < 0.005
    torch.testing.assert_close(y[keep], x.detach()[keep] / (1 - p))
    G = torch.randn_like(y)
    (y * G).sum().backward()
    torch.testing.assert_close(x.grad, torch.where(keep, G / (1 - p), torch.zeros_like(G)))
    y2 = T.dropout(x, p)
    assert ((y2 != 0) != keep).float().mean().item() > 0.2  # fresh mask per call
    T.manual_seed(123)
    assert torch.equal(T.dropout(x, p) != 0, keep)         # reproducible from the seed
    assert T.dropout(x, 0.0) is x


@pytest.mark.gpu
def test_resid_relu_head_gradients_match_oracle():
    """3-layer mapping (two residual blocks) gradient vs the fp64 oracle on random data."""
    from cmve.linas.model import Latent_mapping
    torch.manual_seed(4)
    lm = Latent_mapping([70, 50, 50, 50], 0.0).cuda().train()
    with torch.no_grad():
        for k in (1, 2, 3):
            getattr(lm.mapping, f"fc{k}").bias.normal_(0, 0.3)
    x = torch.randn(33, 70, device="cuda")
    G = torch.randn(33, 50, device="cuda")
    P = {k.replace("mapping.", "").replace("bn_1.", "bn."): v.detach().cpu().numpy()
         for k, v in lm.named_parameters()}
    (lm(x) * G).sum().backward()
    _, tape = OT.mapping_forward(x.cpu().numpy(), P, 3)
    _, gr = OT.mapping_backward(G.cpu().numpy().astype(np.float64), P, 3, tape)
    for k, p in lm.named_parameters():
        kk = k.replace("mapping.", "").replace("bn_1.", "bn.")
        np.testing.assert_allclose(p.grad.cpu().numpy(), gr[kk], rtol=1e-4, atol=5e-6, err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_f32_mfma_is_an_fp32_fma_chain(ta, tb):
    """cmve_gemm_f32[_ex] on v_mfma_f32_16x16x4_f32: ragged M/N/K (tile and K-slab edges), every
    transpose, bias + relu epilogue, beta accumulate; within the fp32 fmaf-chain bound of an fp64
    reference (|err| <= K * 2^-24 * sum|a b|)."""
    from cmve import engine
    from cmve._lib import lib, check
    torch.manual_seed(ta * 2 + tb)
    for M, N, K in [(1, 1, 1), (65, 63, 33), (128, 1024, 1024), (200, 70, 5)]:
        A = torch.randn((K, M) if ta else (M, K), device="cuda")
        Bm = torch.randn((N, K) if tb else (K, N), device="cuda")
        bias = torch.randn(N, device="cuda")
        C0 = torch.randn(M, N, device="cuda")
        Ad, Bd = A.double().T if ta else A.double(), Bm.double().T if tb else Bm.double()
        for relu, beta in ((0, 0.0), (1, 0.5)):
            C = C0.clone()
            check(lib.cmve_gemm_f32_ex(engine.handle(), ta, tb, M, N, K, 0.75, engine._ptr(A), A.stride(0),
                                       engine._ptr(Bm), Bm.stride(0), beta, engine._ptr(C), C.stride(0),
                                       engine._ptr(bias), relu), "cmve_gemm_f32_ex")
            want = 0.75 * (Ad @ Bd) + beta * C0.double() + bias.double()
            if relu:
                want = want.clamp(min=0)
            bound = 0.75 * (Ad.abs() @ Bd.abs()) * K * 2.0 ** -24 + 1e-6 * (1 + want.abs())
            assert bool(((C.double() - want).abs() <= bound).all()), (M, N, K, relu)


@pytest.mark.gpu
def test_c2_scale_steps_track_torch_fp32():
    """At the C2 shape (B = 128, 1024 -> 1024 heads, frames pooled by K2) 24 train_emb steps from
    identical weights follow a plain PyTorch fp32 restatement of the same step (nn.Linear +
    BatchNorm1d + l2norm, loss.py TripletLoss formula, clip_grad_norm_, torch.optim.Adam)."""
    from cmve.linas.model import Latent_mapping, temporal_pool
    from cmve.linas.loss import TripletLoss
    from cmve.linas.train import GTTrainer
    nn = torch.nn
    torch.manual_seed(0)
    B, F, D, T = 128, 1024, 1024, 64

    class Head(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc1, self.bn_1 = nn.Linear(F, D), nn.BatchNorm1d(D)

        def forward(self, x):
            y = self.bn_1(self.fc1(x))
            return y / y.pow(2).sum(1, keepdim=True).sqrt()

    def triplet(s, im, margin=0.2):
        S = im.mm(s.t())
        d = S.diag().view(-1, 1)
        I = torch.eye(S.size(0), device=S.device) > .5
        cs = (margin + S - d.expand_as(S)).clamp(min=0).masked_fill_(I, 0).max(1)[0]
        ci = (margin + S - d.t().expand_as(S)).clamp(min=0).masked_fill_(I, 0).max(0)[0]
        return cs.sum() + ci.sum()

    ref = [Head().cuda().train(), Head().cuda().train()]
    mine = [Latent_mapping([F, D], 0.0).cuda(), Latent_mapping([F, D], 0.0).cuda()]
    with torch.no_grad():
        for a, b in zip(mine, ref):
            a.mapping.fc1.weight.copy_(b.fc1.weight)
            a.mapping.fc1.bias.copy_(b.fc1.bias)
    params = list(ref[0].parameters()) + list(ref[1].parameters())
    opt = torch.optim.Adam(params, lr=1e-4)
    tr = GTTrainer(mine[0], mine[1], TripletLoss(0.2, 'cosine', True, 'sum', 'all'), learning_rate=1e-4,
                   grad_clip=2.0)
    tr.train_start()
    batches = []
    for _ in range(4):
        lengths = torch.randint(20, T + 1, (B,), device="cuda", dtype=torch.int32)
        batches.append((torch.randn(B, T, F, device="cuda"), lengths, torch.randn(B, F, device="cuda")))
    for i in range(24):
        f, l, c = batches[i % 4]
        mask = (torch.arange(T, device="cuda")[None, :] < l[:, None].long()).float()
        pooled_ref = (f * mask[:, :, None]).sum(1) / l[:, None].float()
        pooled = temporal_pool(f, "mean_valid", l)
        torch.testing.assert_close(pooled, pooled_ref, rtol=1e-6, atol=1e-6)
        opt.zero_grad()
        loss_ref = triplet(ref[1](c), ref[0](pooled_ref))
        loss_ref.backward()
        torch.nn.utils.clip_grad_norm_(params, 2.0)
        opt.step()
        _, loss = tr.train_emb(pooled, c)
        np.testing.assert_allclose(loss, float(loss_ref), rtol=2e-4, err_msg=f"step {i}")
    for a, b in zip(mine, ref):
        torch.testing.assert_close(a.mapping.fc1.weight, b.fc1.weight, rtol=0, atol=2e-5)  # Adam on ~0 grads
        torch.testing.assert_close(a.mapping.bn_1.running_var, b.bn_1.running_var, rtol=1e-5, atol=1e-7)


@pytest.mark.gpu
def test_graphed_step_equals_eager_step():
    """GTTrainer(graph=True): warm-up, capture and replays give the same trajectory as eager steps
    from the same weights and dropout seed (device-side dropout position and Adam step count)."""
    from cmve.linas.model import Latent_mapping
    from cmve.linas.loss import TripletLoss
    from cmve.linas import train as T
    torch.manual_seed(2)
    init = [Latent_mapping([96, 64], 0.2).cuda(), Latent_mapping([80, 64, 64], 0.2).cuda()]
    batches = [(torch.randn(32, 96, device="cuda"), torch.randn(32, 80, device="cuda")) for _ in range(3)]
    runs = []
    for graph in (False, True):
        heads = [Latent_mapping([96, 64], 0.2).cuda(), Latent_mapping([80, 64, 64], 0.2).cuda()]
        for h, h0 in zip(heads, init):
            h.load_state_dict(h0.state_dict())
        tr = T.GTTrainer(heads[0], heads[1], TripletLoss(0.2, 'cosine', True, 'sum', 'all'), learning_rate=1e-3,
                         grad_clip=2.0, graph=graph)
        tr.train_start()
        T.manual_seed(77)
        losses = [tr.train_emb(*batches[i % 3])[1] for i in range(7)]
        runs.append((losses, [p.detach().clone() for p in tr.params], heads))
    np.testing.assert_allclose(runs[1][0], runs[0][0], rtol=1e-6)
    for a, b in zip(runs[1][1], runs[0][1]):
        torch.testing.assert_close(a, b, rtol=0, atol=1e-6)
    for ha, hb in zip(runs[1][2], runs[0][2]):
        assert int(ha.mapping.bn_1.num_batches_tracked) == int(hb.mapping.bn_1.num_batches_tracked) == 7
        torch.testing.assert_close(ha.mapping.bn_1.running_var, hb.mapping.bn_1.running_var, rtol=1e-6, atol=0)
