"""LINAS checkpoints and the query encoder built from them.

``load_checkpoint`` reads the reference's ``model_best.pth.tar`` layout (trainer.py:288-293:
{'epoch', 'model': BaseModel.state_dict() slot list, 'best_rsum', 'opt': argparse.Namespace,
'Eiters'}) with ``torch.load(weights_only=True)``: only tensors, containers, the Namespace and numpy
arrays (opt.we_parameter) are admitted -- nothing in the file is executed.  A checkpoint holding
anything else is refused.

``QueryEncoder`` is ``Dual_Encoding.embed_txt_distill`` (model.py:750-781) for a loaded checkpoint:
the student text encoder (or the teacher's, student_model 'map') and the student text mapping,
loaded from the slots BaseModel.load_state_dict(..., 'test') uses (model.py:406-425).
"""
from __future__ import annotations

import argparse
from typing import Optional, Sequence

import numpy as np
import torch

from .. import engine
from .model import Latent_mapping
from . import text as T

# BaseModel.state_dict slots (model.py:387-404)
SLOT_TEXT_ENC, SLOT_TEXT_MAP, SLOT_STUDENT_TEXT_MAP, SLOT_STUDENT_TEXT_ENC = 1, 3, 4, 5


def _safe_globals():
    allowed = [argparse.Namespace, np.ndarray, np.dtype]
    try:  # numpy array reconstruction (numpy 2: numpy._core; numpy 1: numpy.core)
        from numpy._core.multiarray import _reconstruct, scalar
    except ImportError:  # pragma: no cover
        from numpy.core.multiarray import _reconstruct, scalar
    allowed += [_reconstruct, scalar]
    allowed += [type(np.dtype(t)) for t in ("float32", "float64", "int64", "int32", "bool")]
    return allowed


def load_checkpoint(path: str) -> dict:
    """The reference checkpoint dict, through torch's weights-only unpickler (see module doc)."""
    with torch.serialization.safe_globals(_safe_globals()):
        return torch.load(path, map_location="cpu", weights_only=True)


class QueryEncoder:
    """embed_txt_distill (model.py:750-781) on the cmve modules, in eval mode."""

    def __init__(self, opt, model_state: Sequence, device=None):
        self.device = device or engine.default_device()
        self.opt = opt
        student_model = getattr(opt, "student_model", None)
        if student_model == "map":
            enc_cls = T.Text_multilevel_encoding_ori if opt.teacher_model == "student" else T.Text_multilevel_encoding
            enc_slot = SLOT_TEXT_ENC
            layers = list(opt.text_mapping_layers)
        else:
            enc_cls, enc_slot = T.Text_multilevel_encoding_ori, SLOT_STUDENT_TEXT_ENC
            layers = list(opt.text_mapping_layers)
            if student_model == "text+video":  # model.py:568-574: residual blocks appended
                layers += [opt.text_mapping_layers[-1]] * int(getattr(opt, "text_resblock_number", 0))
        self.encoder = enc_cls(opt)
        self.encoder.load_state_dict(model_state[enc_slot])
        self.mapping = Latent_mapping(layers, opt.dropout, getattr(opt, "tag_vocab_size", True))
        self.mapping.load_state_dict(model_state[SLOT_STUDENT_TEXT_MAP])
        self.encoder.to(self.device).eval()
        self.mapping.to(self.device).eval()

    @classmethod
    def from_checkpoint(cls, path: str, device=None) -> "QueryEncoder":
        ck = load_checkpoint(path)
        return cls(ck["opt"], ck["model"], device)

    @torch.no_grad()
    def __call__(self, txt_data) -> torch.Tensor:
        captions, cap_bows, lengths, cap_masks = txt_data
        dev = self.device
        txt = (captions.to(dev) if captions is not None else None,
               cap_bows.to(dev) if cap_bows is not None else None,
               torch.Tensor(list(lengths)) if lengths is not None else None,
               cap_masks.to(dev) if cap_masks is not None else None)
        if isinstance(self.encoder, T.Text_multilevel_encoding):
            return self.mapping(self.encoder(txt, None))
        return self.mapping(self.encoder(txt))

    def encode_captions(self, captions: Sequence[str], vocab: T.Vocabulary, bow2vec: Optional[T.Bow2Vec],
                        batch_size: int = 128) -> np.ndarray:
        """evaluation.encode_text (evaluation.py:119-171) over raw captions: float64 [N, D] in input order."""
        out = None
        for s in range(0, len(captions), batch_size):
            chunk = captions[s:s + batch_size]
            txt, idxs, _ = T.collate_text(chunk, vocab, bow2vec, idxs=range(s, s + len(chunk)), device=self.device)
            emb = self(txt).cpu().numpy()
            if out is None:
                out = np.zeros((len(captions), emb.shape[1]))
            out[list(idxs)] = emb
        return out
