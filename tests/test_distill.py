"""Distillation training step: K15 pair losses, the similarity-distillation variants
and DistillTrainer.train_emb against the reference's own Dual_Encoding.train_emb
(tests/golden/distill.npz, tests/golden/make_golden_distill.py): 9 option sets x 3 steps.

Tolerances: losses rtol 1e-5 (NaN where the reference's KLDivLoss takes the log of a negative target);
first-step (clipped) gradients rtol 1e-4 / atol 1e-4 of the tensor's largest entry; parameters after
3 Adam steps (lr 1e-3) atol 2e-6 for all but 0.5% of the entries and 0.1 lr per step for those few:
Adam divides by the running gradient RMS, so an entry whose gradient nearly cancels turns a 1e-7 fp32
difference into an update difference of a few 1e-5.  The bias of a Linear feeding BatchNorm directly
(fc1.bias of a one-layer head) has an exactly-zero true gradient -- every implementation's is rounding
noise and Adam turns noise into steps of ~lr -- so it (and the BN running mean it shifts) is checked to
within lr per step, as in tests/test_train.py.  The 'svd' case's log-SVD (LAPACK on the host,
as the reference; see cmve.linas.distill._log_svd) amplifies fp32 differences of s2, so its parameters
get atol 2e-5.
"""
import numpy as np
import pytest
import torch

import make_golden_distill as MG

HEADS = MG.HEADS


def test_legacy_reduction_arguments():
    from cmve.linas.distill import MSELoss, SmoothL1Loss, KLDivLoss
    assert MSELoss(reduce=True, size_average=False).reduction == "sum"      # model.py:557
    assert KLDivLoss(reduce=True, size_average=True).reduction == "mean"    # model.py:561
    assert SmoothL1Loss().reduction == "mean"
    with pytest.raises(NotImplementedError):
        SmoothL1Loss(reduce=False)                                          # the elementwise huberloss


@pytest.mark.gpu
@pytest.mark.parametrize("kind,name", [(0, "mse"), (1, "smooth_l1"), (2, "kl")])
@pytest.mark.parametrize("reduction", ["sum", "mean"])
def test_pair_losses_match_torch(kind, name, reduction):
    from cmve.linas import distill as DL
    g = torch.Generator().manual_seed(kind)
    x = (torch.randn(37, 29, generator=g) * 2).cuda().requires_grad_(True)
    y = (torch.randn(37, 29, generator=g) * 2).cuda()
    if kind == 2:
        y = y.abs() + 0.01          # KL over positive targets: finite everywhere
    y.requires_grad_(True)
    mod = {0: DL.MSELoss, 1: DL.SmoothL1Loss, 2: DL.KLDivLoss}[kind](reduction=reduction)
    ref = {0: torch.nn.MSELoss, 1: torch.nn.SmoothL1Loss, 2: torch.nn.KLDivLoss}[kind](reduction=reduction)
    xr, yr = x.detach().clone().requires_grad_(True), y.detach().clone().requires_grad_(True)
    lo, lr_ = mod(x, y), ref(xr, yr)
    torch.testing.assert_close(lo, lr_, rtol=1e-5, atol=1e-6)
    (lo * 1.7).backward()
    (lr_ * 1.7).backward()
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(y.grad, yr.grad, rtol=1e-5, atol=1e-6)  # log(y) + 1 - x cancels near 0
    # torch's NaN semantics: a negative KL target makes the loss NaN, the input gradient stays -target
    if kind == 2:
        yn = torch.tensor([0.5, -0.25, 0.0], device="cuda")
        xn = torch.tensor([0.1, 0.2, 0.3], device="cuda", requires_grad=True)
        ln = DL.KLDivLoss(reduction="sum")(xn, yn)
        assert torch.isnan(ln)
        ln.backward()
        torch.testing.assert_close(xn.grad, -yn)
        # the target gradient where the target is 0 or negative (the reference's model.py:878/880 pass a
        # target that requires grad): torch's kl_div is xlogy(t, t) - t * x, whose autograd gives
        # log(t) + t / t - x -- NaN at t == 0 as well as t < 0 (torch 1.9's fused backward masked t == 0
        # to 0; the goldens are made with this container's torch, which we follow)
        yg = yn.detach().clone().requires_grad_(True)
        DL.KLDivLoss(reduction="sum")(xn.detach(), yg).backward()
        yc = yn.detach().cpu().clone().requires_grad_(True)
        torch.nn.KLDivLoss(reduction="sum")(xn.detach().cpu(), yc).backward()
        torch.testing.assert_close(yg.grad.cpu(), yc.grad, equal_nan=True)


def _heads(g, pre):
    from cmve.linas.model import Latent_mapping
    out = {}
    for h in HEADS:
        key = f"{pre}init.{h}."
        sd = {k[len(key):]: torch.from_numpy(np.asarray(g[k])) for k in g.files if k.startswith(key)}
        if not sd:
            out[h] = None
            continue
        n_lin = sum(1 for k in sd if k.endswith(".weight") and ".fc" in k)
        layers = [sd["mapping.fc1.weight"].shape[1]] + [sd[f"mapping.fc{i}.weight"].shape[0] for i in range(1, n_lin + 1)]
        m = Latent_mapping(layers, 0.0).cuda()
        m.load_state_dict(sd)
        out[h] = m
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(MG.CASES))
def test_distill_train_step_matches_reference(golden, case):
    from cmve.linas.distill import DistillTrainer
    from cmve.linas.loss import TripletLoss
    g = golden("distill")
    pre = f"{case}."
    opt = MG.make_opt(**MG.CASES[case])
    heads = _heads(g, pre)
    crit = TripletLoss(margin=opt.margin, measure=opt.measure, max_violation=opt.max_violation,
                       cost_style=opt.cost_style, direction=opt.direction)
    tr = DistillTrainer(heads["vid_mapping"], heads["text_mapping"], heads["student_text_mapping"],
                        heads["student_vid_mapping"], crit, student_model=opt.student_model,
                        distill_loss=opt.distill_loss, distill_type=opt.distill_type, cost_style=opt.cost_style,
                        alpha=opt.alpha, beta=opt.beta, video_alpha=opt.video_alpha,
                        distill_with_triplet=opt.distill_with_triplet,
                        distill_with_similarity=opt.distill_with_similarity, similarity_type=opt.similarity_type,
                        with_detach=opt.with_detach, finetune_vid=opt.finetune_vid, learning_rate=MG.LR,
                        grad_clip=MG.GRAD_CLIP, mask=torch.from_numpy(g[pre + "mask"]).cuda())
    tr.train_start()
    names = list(g[pre + "param_names"])
    assert len(names) == len(tr.params)
    for t in range(MG.STEPS):
        v, sv = (torch.from_numpy(a).cuda() for a in g[f"{pre}step{t}_feats"])
        c, sc = (torch.from_numpy(a).cuda() for a in g[f"{pre}step{t}_tfeats"])
        if opt.student_model == "text+video":
            ret = tr.train_emb((v, sv), (c, sc))
        else:
            ret = tr.train_emb(v, (c, sc))
        np.testing.assert_allclose(np.array(ret, np.float64), g[f"{pre}step{t}_ret"], rtol=1e-5, atol=1e-6,
                                   equal_nan=True, err_msg=f"{case} step {t}")
        if t == 0:
            for name, p in zip(names, tr.params):
                key = f"{pre}grad0.{name}"
                if key not in g.files:
                    assert p.grad is None, f"{case} {name}: the reference has no gradient here"
                    continue
                want = g[key]
                if name.endswith("mapping.fc1.bias") and f"{pre}init.{name.split('.')[0]}.mapping.fc2.weight" \
                        not in g.files:
                    continue  # zero true gradient (see the module doc)
                np.testing.assert_allclose(p.grad.cpu().numpy(), want, rtol=1e-4,
                                           atol=1e-4 * float(np.abs(want).max()) + 1e-12, err_msg=f"{case} {name}")
    base = 2e-5 if opt.similarity_type == "svd" else 2e-6
    for name, p in zip(names, tr.params):
        h = name.split(".")[0]
        one_layer = f"{pre}init.{h}.mapping.fc2.weight" not in g.files
        got, want = p.detach().cpu().numpy(), g[f"{pre}final.{name}"]
        if one_layer and name.endswith("mapping.fc1.bias"):
            np.testing.assert_allclose(got, want, rtol=0, atol=1.1 * MG.LR * MG.STEPS, err_msg=f"{case} {name}")
            continue
        err = np.abs(got - want)
        assert np.count_nonzero(err > base) <= max(1, 0.005 * err.size), f"{case} {name}: {np.sort(err.ravel())[-5:]}"
        assert err.max() <= 0.1 * MG.LR * MG.STEPS, f"{case} {name}: {err.max()}"
    for h, m in heads.items():
        if m is None:
            continue
        sd = m.state_dict()
        one_layer = f"{pre}init.{h}.mapping.fc2.weight" not in g.files
        np.testing.assert_allclose(sd["mapping.bn_1.running_var"].cpu().numpy(),
                                   g[f"{pre}final.{h}.mapping.bn_1.running_var"], rtol=1e-5, err_msg=h)
        np.testing.assert_allclose(sd["mapping.bn_1.running_mean"].cpu().numpy(),
                                   g[f"{pre}final.{h}.mapping.bn_1.running_mean"],
                                   atol=(0.11 * MG.LR * MG.STEPS if one_layer else 2e-6), err_msg=h)
