"""Golden vectors for the training-step row, produced by running the
REFERENCE's own modules in the build container:

  LINAS-engine/model.py:51-116,362-381   MFC / Latent_mapping in training mode (batch-stat BN)
  LINAS-engine/loss.py:83-153            TripletLoss (margin 0.2, max_violation, sum, all)
  LINAS-engine/model.py:984-1004         train_emb 'GT': zero_grad -> loss -> backward ->
                                         clip_grad_norm_(params, grad_clip) -> Adam.step
  (model.py:481-494 parameter order, :593 torch.optim.Adam)

Dual_Encoding itself needs CUDA and a full option set (model.py:584-588), so the step is driven
here line by line over the reference's mapping heads and loss, with dropout 0 (nn.Dropout draws
from torch's random stream, which no other implementation reproduces).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train.py /root/reference
Writes tests/golden/train_step.npz and tests/golden/train_bn_l2.npz.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))

B, F_VID, F_TXT, D = 32, 96, 80, 64
VID_LAYERS, TXT_LAYERS = [F_VID, D], [F_TXT, D, D]     # text head with one residual block
STEPS, LR, GRAD_CLIP = 3, 1e-3, 2.0


def batches(seed=7):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(B, F_VID, generator=g) * 2.0 + 0.5, torch.randn(B, F_TXT, generator=g)) for _ in range(STEPS)]


def init_heads(M):
    torch.manual_seed(3)
    vm = M.Latent_mapping(VID_LAYERS, 0.0, l2norm=True)
    tm = M.Latent_mapping(TXT_LAYERS, 0.0, l2norm=True)
    for lm in (vm, tm):  # non-trivial affine / biases so every gradient path is exercised
        lm.mapping.bn_1.weight.data.uniform_(0.5, 1.5)
        lm.mapping.bn_1.bias.data.normal_(0, 0.2)
        for k in range(1, len(lm.mapping.__dict__["_modules"])):
            fc = getattr(lm.mapping, f"fc{k}", None)
            if fc is not None:
                fc.bias.data.normal_(0, 0.1)
    return vm, tm


def sd_np(prefix, m):
    return {f"{prefix}{k}": v.detach().numpy().copy() for k, v in m.state_dict().items()}


def main(ref_root):
    sys.path.insert(0, os.path.join(ref_root, "LINAS-engine"))
    import model as M  # noqa
    import loss as L  # noqa
    from torch.nn.utils.clip_grad import clip_grad_norm_

    out = {}
    vm, tm = init_heads(M)
    out.update(sd_np("init_vid.", vm))
    out.update(sd_np("init_txt.", tm))
    vm.train()
    tm.train()
    crit = L.TripletLoss(margin=0.2, measure='cosine', max_violation=True, cost_style='sum', direction='all')
    params = list(vm.parameters()) + list(tm.parameters())
    opt = torch.optim.Adam(params, lr=LR)
    for t, (v, c) in enumerate(batches()):
        out[f"step{t}_videos"] = v.numpy()
        out[f"step{t}_captions"] = c.numpy()
        vid_emb, cap_emb = vm(v), tm(c)                       # forward_emb
        opt.zero_grad()
        loss = crit(cap_emb, vid_emb)                          # forward_loss(cap_emb, vid_emb)
        out[f"step{t}_loss"] = np.array(loss.item())
        loss.backward()
        out[f"step{t}_total_norm"] = np.array(float(clip_grad_norm_(params, GRAD_CLIP)))
        for i, p in enumerate(params):
            out[f"step{t}_grad{i}"] = p.grad.numpy().copy()
        opt.step()
        out[f"step{t}_vid_emb"] = vid_emb.detach().numpy()
        out[f"step{t}_cap_emb"] = cap_emb.detach().numpy()
    out.update(sd_np("final_vid.", vm))
    out.update(sd_np("final_txt.", tm))
    for i, p in enumerate(params):
        st = opt.state[p]
        out[f"adam{i}_exp_avg"] = st["exp_avg"].numpy()
        out[f"adam{i}_exp_avg_sq"] = st["exp_avg_sq"].numpy()
    out["param_names"] = np.array([f"vid.{k}" for k, _ in vm.named_parameters()] +
                                  [f"txt.{k}" for k, _ in tm.named_parameters()])
    np.savez_compressed(os.path.join(HERE, "train_step.npz"), **out)

    # Latent_mapping training forward + backward under a non-uniform upstream gradient
    torch.manual_seed(5)
    lm = M.Latent_mapping([48, 40], 0.0, l2norm=True)
    lm.mapping.bn_1.weight.data.uniform_(0.5, 1.5)
    lm.mapping.bn_1.bias.data.normal_(0, 0.2)
    lm.mapping.fc1.bias.data.normal_(0, 0.1)
    sd0 = sd_np("init.", lm)
    lm.train()
    g = torch.Generator().manual_seed(9)
    x = (torch.randn(20, 48, generator=g) * 3.0 - 1.0).requires_grad_(True)
    G = torch.randn(20, 40, generator=g)
    y = lm(x)
    (y * G).sum().backward()
    bn_out = dict(x=x.detach().numpy(), G=G.numpy(), y=y.detach().numpy(), dx=x.grad.numpy(), **sd0,
                  **{f"grad.{k}": p.grad.numpy() for k, p in lm.named_parameters()}, **sd_np("after.", lm))
    np.savez_compressed(os.path.join(HERE, "train_bn_l2.npz"), **bn_out)
    print(sorted(out)[:8], len(out), sorted(bn_out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
