"""Drop-in mirror of the ``LINAS-engine/inference.py`` gallery scorer + CLI.

Reference hot loop (inference.py:76-82):
    errors = evaluation.cal_error(video_embs, cap_emb, options.measure)   # re-normalises the gallery
    inds = np.argsort(errors[0])[:opt.topK]                               # full O(N log N) sort
    print([video_ids[i] for i in inds])
Here the gallery is normalised and packed into HBM ONCE (``GalleryScorer``) and each
query batch is scored by ``cmve_topk``: a gallery-streaming fp16 MFMA GEMV for up to 32
queries (the GEMM beyond), a histogram bound on the k-th score, and an exact fp64 re-score
of the error band: same ids, same order (score desc; ties by index) as the reference's
argsort on tie-free scores.

CLI (same flags as inference.py:37-44, plus the inputs the frozen encoder would make):
  python -m cmve.linas.inference --input "a man ..." --topK 10 --gpu 0 \
      --gallery video_data.npz --query-emb cap.npy
``--gallery`` is an .npz with ``video_embs`` [N, D] and ``video_ids`` (the content of the
reference's ``video_data.pt`` cache, inference.py:57-67); ``--query-emb`` is the caption
embedding that ``model.embed_txt_distill(process_cap(input))`` produces (inference.py:76-77).
With ``--checkpoint`` (the reference's model_best.pth.tar, loaded weights-only) and the two
vocabularies, ``--input`` is encoded exactly as inference.py:69-77 does (cmve.linas.text.process_cap
-> cmve.linas.checkpoint.QueryEncoder); the reference's own checkpoint
``student_support_set_8/model_best.pth.tar`` is not shipped (LINAS-engine/readme.md:17).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

from .. import engine
from .._lib import SIM_F16


class GalleryScorer:
    """A video gallery resident in HBM, normalised once (LINAS l2norm, no eps)."""

    def __init__(self, video_embs, video_ids=None, with_lo=True):
        emb = video_embs if hasattr(video_embs, "data_ptr") else np.asarray(video_embs)
        self.gallery = engine.RowSet(emb, eps=0.0, with_lo=with_lo)
        self.video_ids = list(video_ids) if video_ids is not None else None
        self._ws = None
        self._q = {}    # resident query sets by (rows, dim, dtype): re-packed in place per call
        self._out = {}  # resident top-k outputs by (rows, k)

    def topk_indices(self, cap_embs, topK=10):
        """[N_q, topK] gallery indices, best first (== np.argsort(cal_error(...)[i])[:topK])."""
        import torch
        if not torch.is_tensor(cap_embs):
            cap_embs = np.atleast_2d(np.asarray(cap_embs))
        elif cap_embs.dim() == 1:
            cap_embs = cap_embs[None, :]
        key = (tuple(cap_embs.shape), str(cap_embs.dtype))
        q = self._q.get(key)
        if q is None:
            q = self._q[key] = engine.RowSet(cap_embs, eps=0.0, with_lo=self.gallery.has_lo,
                                             device=self.gallery.device)
        else:
            q.repack(cap_embs)
        k = min(topK, self.gallery.n)
        need = engine.topk_workspace_floats(q, self.gallery, k)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.float32, device=self.gallery.device)
        out = self._out.get((q.n, k))
        if out is None:
            dev = self.gallery.device
            out = self._out[(q.n, k)] = (torch.empty((max(q.n, 1), k), dtype=torch.int32, device=dev),
                                         torch.empty((max(q.n, 1), k), dtype=torch.float64, device=dev),
                                         torch.zeros(1, dtype=torch.int32, device=dev))
        idx, _ = engine.topk(q, self.gallery, topK, mode=SIM_F16, scores_ws=self._ws, out=out)
        return idx

    def topk_ids(self, cap_emb, topK=10):
        inds = self.topk_indices(cap_emb, topK)[0]
        return [self.video_ids[i] for i in inds]


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--input', default='a man and a woman is talking.', type=str, help='input sentence')
    p.add_argument('--topK', default=10, type=int, help='return top-k videos')
    p.add_argument('--gpu', default='0', type=str, help='gpu device')
    p.add_argument('--gallery', default='video_data.npz', type=str,
                   help='npz with video_embs [N,D] and video_ids (the video_data.pt cache content)')
    p.add_argument('--query-emb', default=None, type=str,
                   help='.npy caption embedding [1,D] (output of the frozen text encoder for --input)')
    p.add_argument('--checkpoint', default=None, type=str,
                   help='LINAS model_best.pth.tar: encode --input with its text encoder + mapping '
                        '(loaded weights-only, cmve.linas.checkpoint)')
    p.add_argument('--rnn-vocab', default=None, type=str, help='rnn vocabulary (.json or the reference .pkl)')
    p.add_argument('--bow-vocab', default=None, type=str, help='bow vocabulary (.json or the reference .pkl)')
    return p.parse_args(argv)


def main(argv=None):
    opt = parse_args(argv)
    os.environ.setdefault("HIP_VISIBLE_DEVICES", opt.gpu)
    if opt.query_emb is None and not (opt.checkpoint and opt.rnn_vocab and opt.bow_vocab):
        sys.exit("cmve inference: give --query-emb, or --checkpoint with --rnn-vocab and --bow-vocab "
                 "(inference.py:49-77: checkpoint + vocabularies -> process_cap -> embed_txt_distill)")
    data = np.load(opt.gallery, allow_pickle=False)
    scorer = GalleryScorer(data['video_embs'], [str(v) for v in data['video_ids']])
    if opt.query_emb is not None:
        cap_emb = np.load(opt.query_emb, allow_pickle=False).astype(np.float32)
    else:
        from .checkpoint import QueryEncoder
        from . import text as T
        enc = QueryEncoder.from_checkpoint(opt.checkpoint)
        vocab, bow_vocab = T.load_vocab(opt.rnn_vocab), T.load_vocab(opt.bow_vocab)
        cap_emb = enc(T.process_cap(opt.input, vocab, T.get_text_encoder('bow')(bow_vocab))).cpu().numpy()
    print(scorer.topk_ids(cap_emb, opt.topK))


if __name__ == '__main__':
    main()
