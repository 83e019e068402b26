"""Golden vectors for the video-side encoder facade and the inference CLI,
produced by running the REFERENCE's own code in the build container:

  LINAS-engine/model.py:119-176,362-381,512-600  Dual_Encoding (Video_multilevel_encoding +
                                                 Latent_mapping, student 'text+video' / 'de+map')
  LINAS-engine/model.py:385-425                  BaseModel.state_dict (the 9-slot checkpoint list)
  LINAS-engine/model.py:707-781                  embed_vis / embed_vis_distill / embed_txt_distill
  LINAS-engine/evaluation.py:88-116              encode_vid over get_vis_data_loader
  LINAS-engine/util/tag_data_provider.py:317-342,503-512  VisDataSet4DualEncoding + collate_frame
  LINAS-engine/inference.py:15-35,76-82          process_cap -> embed_txt_distill -> cal_error -> argsort

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_dual.py /root/reference

Writes tests/golden/dual_<name>.pth.tar (the reference model's state_dict slots + opt, in the
trainer.py:288-293 checkpoint layout; tensors / Namespace / builtins only, so it loads with
torch.load(weights_only=True)) and tests/golden/dual_<name>.npz (the reference's outputs).

The toy gallery is synth.bigfile_toy (40 videos, 96-d frames, 1..80 frames per video).  One
deviation, forced by the reference itself: encode_vid writes ``embeddings[idxs]`` with the tuple
collate_frame returns, which numpy >= 1.23 reads as a multi-dimensional index (IndexError for a
batch of more than 2 videos); the loader handed to it here yields the same indices as a list, so
the rows land where the reference intends.  torch.Tensor.cuda is patched to identity (CPU box).
"""
from __future__ import annotations

import argparse
import os
import pickle
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import synth  # noqa: E402

QUERIES = ["a man and a woman is talking.", "a dog runs on the grass", "zebra quantum", "A DOG plays; with a cat..."]
TOPK = 10
BATCH = 16
FEAT = 96


def dual_opt(vocab_size, bow_dim, student_model, gru_pool):
    v_rnn, v_kn, v_ks = 24, 8, [2, 3, 4]
    t_rnn, t_kn, t_ks = 8, 4, [2, 3, 4]
    vis_dim = 2 * v_rnn + v_kn * len(v_ks) + FEAT
    txt_dim = 2 * t_rnn + t_kn * len(t_ks) + bow_dim
    return argparse.Namespace(
        model="dual_encoding_latent", grad_clip=2.0, dropout=0.2, concate="full", gru_pool=gru_pool,
        tag_vocab_size=512, loss_fun="mrl", margin=0.2, measure="cosine", max_violation=True, cost_style="sum",
        direction="all", style="distill_from_best_model", student_model=student_model, teacher_model="teacher",
        alpha=0.5, beta=0.5, video_alpha=0.5, distill_type="feat", similarity_type="none",
        distill_with_triplet=True, text_resblock_number=1, batch_size=8, optimizer="adam", learning_rate=1e-4,
        visual_feat_dim=FEAT, visual_rnn_size=v_rnn, visual_kernel_num=v_kn, visual_kernel_sizes=v_ks,
        visual_mapping_layers=[vis_dim, 32], word_dim=16, we_parameter=None, text_rnn_size=t_rnn,
        vocab_size=vocab_size, text_kernel_num=t_kn, text_kernel_sizes=t_ks, text_mapping_layers=[txt_dim, 32],
        hidden_size=10, vocab="word_vocab_5", collections_pathname={"train": "toytrain", "test": "toytest"},
        visual_feature="toyfeat", workers=0)


class _ListIdxLoader:
    """The reference DataLoader with idxs as a list (see the module doc)."""

    def __init__(self, loader):
        self.loader = loader
        self.dataset = loader.dataset

    def __iter__(self):
        for datas, idxs, ids in self.loader:
            yield datas, list(idxs), ids


def _perturb_bn(module, g):
    for m in module.modules():
        if isinstance(m, torch.nn.BatchNorm1d):
            m.running_mean.normal_(0, 0.3, generator=g)
            m.running_var.uniform_(0.5, 2.0, generator=g)
            m.weight.data.uniform_(0.5, 1.5, generator=g)
            m.bias.data.normal_(0, 0.2, generator=g)
        if isinstance(m, torch.nn.Linear) and m.bias is not None:
            m.bias.data.normal_(0, 0.1, generator=g)


def main(ref_root):
    sys.path.insert(0, os.path.join(ref_root, "LINAS-engine"))
    torch.Tensor.cuda = lambda self, *a, **k: self
    import model as M  # noqa
    import evaluation as E  # noqa
    import inference as INF  # noqa  (script body is under __main__)
    from basic.bigfile import BigFile  # noqa
    from basic.util import read_dict  # noqa
    from util import tag_data_provider as TDP  # noqa
    from util import text2vec as T2V  # noqa

    with open(os.path.join(HERE, "text_rnn_vocab.pkl"), "rb") as f:
        rnn_vocab = pickle.load(f)  # written by make_golden_text.py (the reference's own Vocabulary)
    with open(os.path.join(HERE, "text_bow_vocab.pkl"), "rb") as f:
        bow_vocab = pickle.load(f)
    INF.vocab = rnn_vocab
    INF.bow2vec = T2V.get_text_encoder("bow")(bow_vocab)

    for name, student_model, pool, seed in (("tv", "text+video", "max", 11), ("dm", "de+map", "mean", 12)):
        torch.manual_seed(seed)
        opt = dual_opt(len(rnn_vocab), INF.bow2vec.ndims, student_model, pool)
        model = M.get_model(opt.model)(opt)
        g = torch.Generator().manual_seed(seed)
        for attr in ("vid_mapping", "text_mapping", "student_text_mapping", "student_vid_mapping"):
            if hasattr(model, attr):
                _perturb_bn(getattr(model, attr), g)
        model.val_start()
        ck = {"epoch": 3, "model": model.state_dict(), "best_rsum": 1.5, "opt": opt, "Eiters": 42}
        torch.save(ck, os.path.join(HERE, f"dual_{name}.pth.tar"))
        out = {}
        with tempfile.TemporaryDirectory() as d:
            synth.bigfile_toy(d, dim=FEAT)
            bf = BigFile(d)
            v2f = read_dict(os.path.join(d, "video2frames.txt"))
            loader = TDP.get_vis_data_loader(bf, BATCH, 0, v2f, video_ids=list(v2f.keys()))
            with torch.no_grad():
                embs, ids = E.encode_vid(model.embed_vis_distill, _ListIdxLoader(loader))
                teacher = E.encode_vid(model.embed_vis, _ListIdxLoader(loader), return_ids=False)
        out["video_ids"] = np.array(ids)
        out["video_embs"] = embs
        out["video_embs_teacher"] = teacher
        for q, s in enumerate(QUERIES):
            with torch.no_grad():
                cap_emb = model.embed_txt_distill(INF.process_cap(s)).data.cpu().numpy()
            errors = E.cal_error(embs, cap_emb, opt.measure)          # inference.py:78-80
            inds = np.argsort(errors[0])[:TOPK]
            out[f"q{q}_cap_emb"] = cap_emb
            out[f"q{q}_inds"] = inds
            out[f"q{q}_results"] = np.array([ids[i] for i in inds])
        np.savez_compressed(os.path.join(HERE, f"dual_{name}.npz"), **out)
        print("wrote dual_%s" % name, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
