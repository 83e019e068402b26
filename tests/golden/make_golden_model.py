"""Golden vectors for the pool / projection / loss rows (SURVEY 8c items iii-vii), produced by
running the REFERENCE's own modules in the build container:

  LINAS-engine/util/tag_data_provider.py:91-109   collate_frame
  LINAS-engine/model.py:119-176                   Video_multilevel_encoding.forward (gru_pool max / mean)
  LINAS-engine/model.py:51-116,362-381            MFC / Latent_mapping (eval)
  LINAS-engine/loss.py:83-153                     TripletLoss forward + autograd grads
  torch CrossEntropyLoss on 100 * P @ T^T          MultiFusion/src/combiner_train.py:318,367-372 (+ transpose)

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_model.py /root/reference
Writes tests/golden/model_*.npz.  torch.Tensor.cuda is patched to identity while the
reference's CUDA-only lines run (model.py:153 allocates with .cuda()).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main(ref_root):
    sys.path.insert(0, os.path.join(ref_root, "LINAS-engine"))
    import model as M  # noqa
    import loss as L  # noqa
    from util import tag_data_provider as TDP  # noqa
    torch.Tensor.cuda = lambda self, *a, **k: self  # CPU-only container: keep tensors where they are

    out = {}
    # ---- (vi) collate_frame on ragged T (incl. > 64) ----
    g = torch.Generator().manual_seed(0)
    Ts = [3, 64, 70, 100, 17]
    F = 48
    frames = [torch.randn(T, F, generator=g) for T in Ts]
    (vids, origin, lengths, mask), idxs, ids = TDP.collate_frame([(f, i, f"v{i}") for i, f in enumerate(frames)])
    out["collate"] = dict(frames=torch.cat(frames).numpy(), T=np.array(Ts), videos=vids.numpy(),
                          origin=origin.numpy(), lengths=np.array(lengths), mask=mask.numpy())

    # ---- (vii) Video_multilevel_encoding pools (gru_pool max and mean) ----
    for pool in ("max", "mean"):
        torch.manual_seed(1)
        opt = argparse.Namespace(visual_rnn_size=32, dropout=0.2, concate="full", gru_pool=pool, tag_vocab_size=512,
                                 loss_fun="mrl", visual_feat_dim=F, visual_kernel_num=16,
                                 visual_kernel_sizes=[2, 3, 4, 5])
        enc = M.Video_multilevel_encoding(opt).eval()
        with torch.no_grad():
            gru_init_out, _ = enc.rnn(vids)
            feats = enc((vids, origin, lengths, mask))
        sd = {f"sd_{k}": v.numpy() for k, v in enc.state_dict().items()}
        out[f"venc_{pool}"] = dict(gru_init_out=gru_init_out.numpy(), features=feats.numpy(), **sd)

    # ---- (v) Latent_mapping eval forward, plain and with residual layers ----
    for name, layers in (("map2", [512, 256]), ("map3", [256, 256, 256])):
        torch.manual_seed(2)
        lm = M.Latent_mapping(layers, 0.2, l2norm=True)
        bn = lm.mapping.bn_1
        bn.running_mean.normal_(0, 0.3)
        bn.running_var.uniform_(0.5, 2.0)
        bn.weight.data.uniform_(0.5, 1.5)
        bn.bias.data.normal_(0, 0.2)
        for k in range(1, len(layers)):
            getattr(lm.mapping, f"fc{k}").bias.data.normal_(0, 0.1)
        lm.eval()
        x = torch.randn(70, layers[0], generator=g)
        with torch.no_grad():
            y = lm(x)
        sd = {f"sd_{k}": v.numpy() for k, v in lm.state_dict().items()}
        out[f"latent_{name}"] = dict(x=x.numpy(), y=y.numpy(), layers=np.array(layers), **sd)

    # ---- (iii) TripletLoss value + grads ----
    cases = [("mv_sum_all", 0.2, True, "sum", "all", 128), ("mv_sum_all_b8", 0.2, True, "sum", "all", 8),
             ("mv_mean_all", 0.2, True, "mean", "all", 64), ("sum_all", 0.2, False, "sum", "all", 32),
             ("mv_sum_t2v", 0.2, True, "sum", "t2v", 32), ("mv_sum_v2t", 0.2, True, "sum", "v2t", 32),
             ("mean_all", 0.3, False, "mean", "all", 16)]
    for name, m, mv, cs, dr, B in cases:
        gg = torch.Generator().manual_seed(B + len(name))
        s = torch.nn.functional.normalize(torch.randn(B, 96, generator=gg), dim=1).requires_grad_(True)
        im = torch.nn.functional.normalize(torch.randn(B, 96, generator=gg), dim=1).requires_grad_(True)
        crit = L.TripletLoss(margin=m, measure='cosine', max_violation=mv, cost_style=cs, direction=dr)
        loss = crit(s, im)
        loss.backward()
        out[f"triplet_{name}"] = dict(s=s.detach().numpy(), im=im.detach().numpy(), loss=np.array(loss.item()),
                                      ds=s.grad.numpy(), dim=im.grad.numpy(),
                                      cfg=np.array([m, float(mv), float(cs == 'mean'), {"v2t": 1, "t2v": 2, "all": 3}[dr]]))

    # ---- (iv) InfoNCE: row CE on 100 * P @ T^T, col CE on the transpose ----
    for B, D in ((64, 640), (256, 128)):
        gg = torch.Generator().manual_seed(B)
        P = torch.nn.functional.normalize(torch.randn(B, D, generator=gg), dim=-1).requires_grad_(True)
        T = torch.nn.functional.normalize(torch.randn(B, D, generator=gg), dim=-1).requires_grad_(True)
        ce = torch.nn.CrossEntropyLoss()
        gt = torch.arange(B)
        logits = 100 * P @ T.T
        row = ce(logits, gt)
        row.backward(retain_graph=True)
        dP_row, dT_row = P.grad.clone(), T.grad.clone()
        P.grad = None
        T.grad = None
        col = ce(logits.T, gt)
        col.backward()
        out[f"infonce_{B}"] = dict(P=P.detach().numpy(), T=T.detach().numpy(), row=np.array(row.item()),
                                   col=np.array(col.item()), dP_row=dP_row.numpy(), dT_row=dT_row.numpy(),
                                   dP_col=P.grad.numpy(), dT_col=T.grad.numpy())

    for name, d in out.items():
        path = os.path.join(HERE, f"model_{name}.npz")
        np.savez_compressed(path, **{k: np.asarray(v) for k, v in d.items()})
        print("wrote", path, os.path.getsize(path))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
