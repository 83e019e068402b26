"""Golden vectors for the distillation training step, produced by running the
REFERENCE's own Dual_Encoding.train_emb (LINAS-engine/model.py:916-982) in the build container:

  model.py:512-600    Dual_Encoding built from a full option set (style 'distill_from_best_model',
                      student 'text+video' / 'de+map' / 'map'), torch.optim.Adam over init_info's params
  model.py:845-889    forward_loss_distill_similarity (SmoothL1 / 'diag' / 'adapt' / 'maxdiag' / 'svd')
                      and forward_loss_distill (mse / kl / mse+kl / cross)
  model.py:916-982    train_emb: the loss combination, the missing zero_grad of the 'text+video'
                      branch, clip_grad_norm_, Adam.step

The encoders are the frozen backbones on the cmve side, so forward_emb (model.py:600-698) is replaced
here by the same mapping calls on encoder FEATURES (the reference's own Latent_mapping modules, in
train mode); everything after forward_emb is the reference's code.  dropout 0 (nn.Dropout draws from
torch's random stream).  model.mask (model.py:588, all ones at init) is replaced by a seeded matrix so
the 'adapt' weights are not uniform.  torch.Tensor.cuda is patched to identity (CPU box).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_distill.py /root/reference
Writes tests/golden/distill.npz.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
B, FV, FT, D = 16, 48, 40, 32
STEPS, LR, GRAD_CLIP = 3, 1e-3, 2.0
HEADS = ("vid_mapping", "text_mapping", "student_text_mapping", "student_vid_mapping")

# name -> option overrides (model.py option names)
CASES = {
    "tv_all": dict(student_model="text+video", distill_loss="text+video", distill_type="mse", cost_style="sum",
                   distill_with_triplet=True, distill_with_similarity=True, similarity_type="none"),
    "tv_mean_diag_msekl": dict(student_model="text+video", distill_loss="text+video", distill_type="mse+kl",
                               cost_style="mean", distill_with_triplet=True, distill_with_similarity=True,
                               similarity_type="diag"),
    "tv_adapt_video": dict(student_model="text+video", distill_loss="video", distill_type="mse", cost_style="sum",
                           distill_with_triplet=False, distill_with_similarity=True, similarity_type="adapt"),
    "tv_maxdiag_cross": dict(student_model="text+video", distill_loss="text+video", distill_type="cross",
                             cost_style="sum", distill_with_triplet=True, distill_with_similarity=True,
                             similarity_type="maxdiag"),
    "tv_svd_text": dict(student_model="text+video", distill_loss="text", distill_type="mse", cost_style="sum",
                        distill_with_triplet=False, distill_with_similarity=True, similarity_type="svd"),
    "tv_plain": dict(student_model="text+video", distill_loss="text+video", distill_type="mse", cost_style="sum",
                     distill_with_triplet=False, distill_with_similarity=False, similarity_type="none"),
    "dm_nodetach": dict(student_model="de+map", distill_type="mse", cost_style="sum", distill_with_triplet=True,
                        with_detach=False, finetune_vid=False),
    "map_detach": dict(student_model="map", distill_type="mse", cost_style="mean", distill_with_triplet=True,
                       with_detach=True, finetune_vid=False),
    "map_detach_finetune": dict(student_model="map", distill_type="mse", cost_style="sum",
                                distill_with_triplet=True, with_detach=True, finetune_vid=True),
}


def make_opt(**kw):
    o = dict(model="dual_encoding_latent", grad_clip=GRAD_CLIP, dropout=0.0, concate="full", gru_pool="max",
             tag_vocab_size=512, loss_fun="mrl", margin=0.2, measure="cosine", max_violation=True, cost_style="sum",
             direction="all", style="distill_from_best_model", teacher_model="teacher", alpha=0.7, beta=0.3,
             video_alpha=0.5, distill_type="mse", similarity_type="none", distill_with_triplet=True,
             distill_with_similarity=False, distill_loss="text+video", text_resblock_number=1, batch_size=B,
             optimizer="adam", learning_rate=LR, visual_feat_dim=24, visual_rnn_size=8, visual_kernel_num=4,
             visual_kernel_sizes=[2, 3], visual_mapping_layers=[FV, D], word_dim=16, we_parameter=None,
             text_rnn_size=8, vocab_size=30, text_kernel_num=4, text_kernel_sizes=[2, 3],
             text_mapping_layers=[FT, D], hidden_size=10, with_detach=False, finetune_vid=False)
    o.update(kw)
    return argparse.Namespace(**o)


def features(seed, step):
    g = torch.Generator().manual_seed(1000 * seed + step)
    return (torch.randn(B, FV, generator=g) * 1.5 + 0.3, torch.randn(B, FT, generator=g),
            torch.randn(B, FV, generator=g) + 0.2, torch.randn(B, FT, generator=g) * 0.8)


class _Log:
    def update(self, *a, **k):
        pass


def main(ref_root):
    sys.path.insert(0, os.path.join(ref_root, "LINAS-engine"))
    torch.Tensor.cuda = lambda self, *a, **k: self
    import model as M  # noqa
    out = {}
    for ci, (name, kw) in enumerate(CASES.items()):
        torch.manual_seed(100 + ci)
        opt = make_opt(**kw)
        model = M.get_model(opt.model)(opt)
        g = torch.Generator().manual_seed(200 + ci)
        for h in HEADS:
            if hasattr(model, h):
                for m in getattr(model, h).modules():
                    if isinstance(m, torch.nn.BatchNorm1d):
                        m.weight.data.uniform_(0.5, 1.5, generator=g)
                        m.bias.data.normal_(0, 0.2, generator=g)
                    if isinstance(m, torch.nn.Linear):
                        m.bias.data.normal_(0, 0.1, generator=g)
        model.mask = torch.rand(B, B, generator=g) * 2.0
        model.logger = _Log()
        pre = f"{name}."
        out[pre + "mask"] = model.mask.numpy()
        for h in HEADS:
            if hasattr(model, h):
                for k, v in getattr(model, h).state_dict().items():
                    out[f"{pre}init.{h}.{k}"] = v.numpy().copy()
        names = []
        for h in HEADS:
            if hasattr(model, h):
                names += [f"{h}.{k}" for k, _ in getattr(model, h).named_parameters()]
        out[pre + "param_names"] = np.array(names)

        def forward_emb(videos, captions, support, volatile=False, *a):
            v, sv = videos
            c, sc = captions
            vid = model.vid_mapping(v)
            cap = model.text_mapping(c)
            if opt.student_model == "text+video":
                return vid, cap, model.student_vid_mapping(sv), model.student_text_mapping(sc)
            return vid, cap, model.student_text_mapping(sc)
        model.forward_emb = forward_emb
        model.train_start()
        for t in range(STEPS):
            v, c, sv, sc = features(ci, t)
            out[f"{pre}step{t}_feats"] = np.stack([v.numpy(), sv.numpy()])
            out[f"{pre}step{t}_tfeats"] = np.stack([c.numpy(), sc.numpy()])
            ret = model.train_emb(t, (v, sv), (c, sc), None)
            out[f"{pre}step{t}_ret"] = np.array([float(x) for x in ret])
            if t == 0:  # the (clipped) gradients the first Adam step consumed; None = no gradient
                for h in HEADS:
                    if hasattr(model, h):
                        for k, prm in getattr(model, h).named_parameters():
                            if prm.grad is not None:
                                out[f"{pre}grad0.{h}.{k}"] = prm.grad.numpy().copy()
        for h in HEADS:
            if hasattr(model, h):
                for k, v in getattr(model, h).state_dict().items():
                    out[f"{pre}final.{h}.{k}"] = v.numpy().copy()
        print(name, [out[f"{pre}step{t}_ret"] for t in range(STEPS)])
    path = os.path.join(HERE, "distill.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
