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

CLI (same flags and flow as inference.py:37-82; run from the directory that holds the
reference's ``student_support_set_8/`` and ``dataset/``):
  python -m cmve.linas.inference --input "a man ..." --topK 10 --gpu 0
  1. checkpoint ``student_support_set_8/model_best.pth.tar`` -> get_model(opt.model)(opt),
     load_state_dict(checkpoint['model'], 'test'), val_start (weights-only load, cmve.linas.checkpoint)
  2. gallery: ``video_data.pt`` if it exists (weights-only), else BigFile features of
     dataset/<test collection>/FeatureData/<visual_feature> + video2frames.txt -> encode_vid(
     model.embed_vis_distill, ...) on the GPU, written back to ``video_data.pt``
  3. vocabularies dataset/<train collection>/TextData/vocabulary/{bow,rnn}/<vocab>.pkl (restricted
     unpickler) -> process_cap(--input) -> embed_txt_distill
  4. exact top-K of the cosine errors on HBM (GalleryScorer), printed as the id list
``--gpu`` is exported as HIP_VISIBLE_DEVICES before the GPU is touched (the reference's
CUDA_VISIBLE_DEVICES, inference.py:47); its default is '0' rather than the reference's '5', which
would hide every GPU of a box with fewer than six.  ``--query-emb`` (a .npy caption embedding)
and ``--gallery`` (an .npz with video_embs / video_ids) bypass steps 3 and 1-2 respectively.
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
    p.add_argument('--checkpoint', default='student_support_set_8/model_best.pth.tar', type=str,
                   help='LINAS model_best.pth.tar (inference.py:49), loaded weights-only')
    p.add_argument('--rootpath', default='dataset/', type=str, help='dataset root (inference.py:55)')
    p.add_argument('--video-cache', default='video_data.pt', type=str,
                   help='gallery cache {video_embs, video_ids} (inference.py:57-67)')
    p.add_argument('--gallery', default=None, type=str,
                   help='.npz with video_embs [N,D] and video_ids instead of the cache / BigFile')
    p.add_argument('--query-emb', default=None, type=str,
                   help='.npy caption embedding [1,D] instead of encoding --input')
    p.add_argument('--rnn-vocab', default=None, type=str, help='rnn vocabulary (default: the checkpoint opt path)')
    p.add_argument('--bow-vocab', default=None, type=str, help='bow vocabulary (default: the checkpoint opt path)')
    return p.parse_args(argv)


def _gallery(opt, model, options):
    """inference.py:57-67: the video_data.pt cache, else encode_vid over the BigFile features."""
    from . import bigfile as B
    if opt.gallery is not None:
        data = np.load(opt.gallery, allow_pickle=False)
        return data['video_embs'], [str(v) for v in data['video_ids']]
    if os.path.exists(opt.video_cache):
        return B.load_video_cache(opt.video_cache)
    if model is None:
        sys.exit("cmve inference: no gallery (give --gallery, a %s cache, or the checkpoint)" % opt.video_cache)
    from .evaluation import encode_vid
    feat_dir = os.path.join(opt.rootpath, options.collections_pathname['test'], 'FeatureData', options.visual_feature)
    visual_feats = B.BigFile(feat_dir)
    video2frames = B.read_dict(os.path.join(feat_dir, 'video2frames.txt'))
    loader = B.VideoBatchLoader(visual_feats, video2frames, video_ids=list(video2frames.keys()),
                                batch_size=options.batch_size, device=model.device)
    video_embs, video_ids = encode_vid(model.embed_vis_distill, loader)
    B.save_video_cache(opt.video_cache, video_embs, video_ids)
    return video_embs, video_ids


def main(argv=None):
    opt = parse_args(argv)
    os.environ["HIP_VISIBLE_DEVICES"] = opt.gpu
    model = options = None
    if opt.query_emb is None or (opt.gallery is None and not os.path.exists(opt.video_cache)):
        from .checkpoint import load_checkpoint, get_model
        checkpoint = load_checkpoint(opt.checkpoint)
        options = checkpoint['opt']
        model = get_model(options.model)(options)
        model.load_state_dict(checkpoint['model'], 'test')
        model.Eiters = checkpoint['Eiters']
        model.val_start()
    video_embs, video_ids = _gallery(opt, model, options)
    if opt.query_emb is not None:
        cap_emb = np.load(opt.query_emb, allow_pickle=False).astype(np.float32)
    else:
        from . import text as T
        voc = os.path.join(opt.rootpath, options.collections_pathname['train'], 'TextData', 'vocabulary')
        bow_vocab = T.load_vocab(opt.bow_vocab or os.path.join(voc, 'bow', options.vocab + '.pkl'))
        vocab = T.load_vocab(opt.rnn_vocab or os.path.join(voc, 'rnn', options.vocab + '.pkl'))
        bow2vec = T.get_text_encoder('bow')(bow_vocab)
        cap_emb = model.embed_txt_distill(T.process_cap(opt.input, vocab, bow2vec)).cpu().numpy()
    measure = getattr(options, 'measure', 'cosine') if options is not None else 'cosine'
    if measure == 'cosine':
        results = GalleryScorer(video_embs, [str(v) for v in video_ids]).topk_ids(cap_emb, opt.topK)
    else:  # inference.py:78-80 with a cdist / jaccard measure: the all-pairs kernel, then argsort
        from .evaluation import cal_error
        errors = np.asarray(cal_error(video_embs, cap_emb, measure))
        results = [video_ids[i] for i in np.argsort(errors[0])[:opt.topK]]
    print(results)
    return results


if __name__ == '__main__':
    main()
