"""LINAS checkpoints and the query encoder built from them.

``load_checkpoint`` reads the reference's ``model_best.pth.tar`` layout (trainer.py:288-293:
{'epoch', 'model': BaseModel.state_dict() slot list, 'best_rsum', 'opt': argparse.Namespace,
'Eiters'}) with ``torch.load(weights_only=True)``: only tensors, containers, the Namespace and numpy
arrays (opt.we_parameter) are admitted -- nothing in the file is executed.  A checkpoint holding
anything else is refused.

``QueryEncoder`` is ``Dual_Encoding.embed_txt_distill`` (model.py:750-781) for a loaded checkpoint:
the student text encoder (or the teacher's, student_model 'map') and the student text mapping,
loaded from the slots BaseModel.load_state_dict(..., 'test') uses (model.py:406-425).

``Dual_Encoding`` / ``get_model`` are the inference surface of the reference's model class
(model.py:385-425,512-600,707-800,1007-1011): the same modules and attribute names, the 9-slot
``state_dict`` / ``load_state_dict(state, teacher_model)``, ``val_start`` and the ``embed_vis`` /
``embed_vis_distill`` / ``embed_txt_distill`` / ``embed_txt_GT`` encoders, so inference.py's
``get_model(options.model)(options); model.load_state_dict(checkpoint['model'], 'test')`` runs
unchanged.  The training step (forward_emb / train_emb) is cmve.linas.train.
"""
from __future__ import annotations

import argparse
from typing import Optional, Sequence

import numpy as np
import torch

from .. import engine
from .model import Latent_mapping, Video_multilevel_encoding
from . import text as T

# BaseModel.state_dict slots (model.py:387-404)
SLOT_VID_ENC, SLOT_TEXT_ENC, SLOT_VID_MAP, SLOT_TEXT_MAP = 0, 1, 2, 3
SLOT_STUDENT_TEXT_MAP, SLOT_STUDENT_TEXT_ENC, SLOT_STUDENT_VID_MAP, SLOT_STUDENT_VID_ENC = 4, 5, 6, 7


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


def _to(x, dev):
    return x.to(dev) if torch.is_tensor(x) else x


class Dual_Encoding:
    """The reference's Dual_Encoding (model.py:512-600) for inference: modules built from ``opt``,
    loaded by slot, run in eval mode on the cmve kernels (see the module doc)."""

    _MODULES = ("vid_encoding", "text_encoding", "vid_mapping", "text_mapping", "student_text_mapping",
                "student_text_encoding", "student_vid_mapping", "student_vid_encoding")

    def __init__(self, opt, device=None):
        self.device = device or engine.default_device()
        self.opt = opt
        l2 = getattr(opt, "tag_vocab_size", True)
        self.vid_encoding = Video_multilevel_encoding(opt)
        self.vid_mapping = Latent_mapping(opt.visual_mapping_layers, opt.dropout, l2)
        if opt.teacher_model == "student":
            self.text_encoding = T.Text_multilevel_encoding_ori(opt)
        else:
            self.text_encoding = T.Text_multilevel_encoding(opt)
        self.text_mapping = Latent_mapping(opt.text_mapping_layers, opt.dropout, l2)
        self.style = opt.style
        self.student_model = getattr(opt, "student_model", None)
        if self.style == "distill_from_best_model":  # model.py:560-580
            if self.student_model == "map":
                self.student_text_mapping = Latent_mapping(opt.text_mapping_layers, opt.dropout, l2)
            elif self.student_model == "de+map":
                self.student_text_encoding = T.Text_multilevel_encoding_ori(opt)
                self.student_text_mapping = Latent_mapping(opt.text_mapping_layers, opt.dropout, l2)
            elif self.student_model == "text+video":
                self.student_text_encoding = T.Text_multilevel_encoding_ori(opt)
                layers = list(opt.text_mapping_layers)
                layers += [opt.text_mapping_layers[-1]] * int(getattr(opt, "text_resblock_number", 0))
                self.student_text_mapping = Latent_mapping(layers, opt.dropout, l2)
                self.student_vid_encoding = Video_multilevel_encoding(opt)
                self.student_vid_mapping = Latent_mapping(opt.visual_mapping_layers, opt.dropout, l2)
        for m in self._modules():
            m.to(self.device)
        self.Eiters = 0

    def _modules(self):
        return [getattr(self, n) for n in self._MODULES if hasattr(self, n)]

    def state_dict(self):
        """The 9-slot list of model.py:387-404."""
        slots = [None] * 9
        for i, n in enumerate(self._MODULES):
            if hasattr(self, n):
                slots[i] = getattr(self, n).state_dict()
        return slots

    def load_state_dict(self, state_dict, teacher_model):
        """model.py:406-425: 'student' reads the student slots into the teacher modules; anything
        else reads slots 0-3 and the student slots that exist."""
        if teacher_model == "student":
            self.text_mapping.load_state_dict(state_dict[SLOT_STUDENT_TEXT_MAP])
            self.text_encoding.load_state_dict(state_dict[SLOT_STUDENT_TEXT_ENC])
            self.vid_mapping.load_state_dict(state_dict[SLOT_STUDENT_VID_MAP])
            self.vid_encoding.load_state_dict(state_dict[SLOT_STUDENT_VID_ENC])
            return
        self.vid_encoding.load_state_dict(state_dict[SLOT_VID_ENC])
        self.text_encoding.load_state_dict(state_dict[SLOT_TEXT_ENC])
        self.vid_mapping.load_state_dict(state_dict[SLOT_VID_MAP])
        self.text_mapping.load_state_dict(state_dict[SLOT_TEXT_MAP])
        for slot, n in ((SLOT_STUDENT_TEXT_MAP, "student_text_mapping"), (SLOT_STUDENT_TEXT_ENC, "student_text_encoding"),
                        (SLOT_STUDENT_VID_MAP, "student_vid_mapping"), (SLOT_STUDENT_VID_ENC, "student_vid_encoding")):
            if hasattr(self, n) and len(state_dict) > slot and state_dict[slot] is not None:
                getattr(self, n).load_state_dict(state_dict[slot])

    def val_start(self):
        for m in self._modules():
            m.eval()

    @classmethod
    def from_checkpoint(cls, path: str, teacher_model: str = "test", device=None) -> "Dual_Encoding":
        """inference.py:49-54: build from checkpoint['opt'], load checkpoint['model'], eval mode."""
        ck = load_checkpoint(path)
        model = cls(ck["opt"], device)
        model.load_state_dict(ck["model"], teacher_model)
        model.Eiters = ck.get("Eiters", 0)
        model.val_start()
        return model

    def _vis(self, vis_data):
        frames, mean_origin, video_lengths, videos_mask = vis_data
        return (_to(frames, self.device).float(), _to(mean_origin, self.device).float(), video_lengths,
                _to(videos_mask, self.device).float())

    def _txt(self, txt_data):
        captions, cap_bows, lengths, cap_masks = txt_data
        return (_to(captions, self.device), _to(cap_bows, self.device),
                torch.as_tensor(np.asarray(lengths), dtype=torch.float32) if lengths is not None else None,
                _to(cap_masks, self.device))

    @torch.no_grad()
    def embed_vis(self, vis_data, volatile=True):
        """model.py:707-725: vid_mapping(vid_encoding(frames, mean_origin, lengths, mask))."""
        return self.vid_mapping(self.vid_encoding(self._vis(vis_data)))

    @torch.no_grad()
    def embed_vis_distill(self, vis_data, volatile=True):
        """model.py:727-748: the student video branch for student_model 'text+video'."""
        if self.student_model == "text+video":
            return self.student_vid_mapping(self.student_vid_encoding(self._vis(vis_data)))
        return self.vid_mapping(self.vid_encoding(self._vis(vis_data)))

    @torch.no_grad()
    def embed_txt_distill(self, txt_data, volatile=True):
        """model.py:750-781."""
        txt = self._txt(txt_data)
        if self.student_model == "map":
            return self.student_text_mapping(self.text_encoding(txt, None))
        return self.student_text_mapping(self.student_text_encoding(txt))

    @torch.no_grad()
    def embed_txt_GT(self, txt_data, support_txt_data, volatile=True):
        """model.py:783-830: text_mapping(text_encoding(txt, support)) (style 'GT')."""
        return self.text_mapping(self.text_encoding(self._txt(txt_data), self._txt(support_txt_data)))


NAME_TO_MODELS = {"dual_encoding_latent": Dual_Encoding}  # model.py:1007


def get_model(name):
    """model.py:1009-1011."""
    assert name in NAME_TO_MODELS, "%s not supported." % name
    return NAME_TO_MODELS[name]
