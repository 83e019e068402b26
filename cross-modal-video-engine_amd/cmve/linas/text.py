"""Query side of the LINAS retrieval path: tokeniser, vocabularies, BoW, caption
collation and the text encoders, with the pools on libcmve.so.

  clean_str / Vocabulary            LINAS-engine/util/vocab.py:15-35,47-49
  build_vocab                       LINAS-engine/util/vocab.py:60-88
  Bow2Vec                           LINAS-engine/util/text2vec.py:8-74
  process_cap                       LINAS-engine/inference.py:15-35   (one caption -> encoder input)
  collate_text                      LINAS-engine/util/tag_data_provider.py:160-184 (collate_text_distill)
  Text_multilevel_encoding_ori      LINAS-engine/model.py:191-260
  Text_multilevel_encoding          LINAS-engine/model.py:263-359     (support-set gating, style 'GT' /
                                                                       'distill_from_best_model')

The encoders keep the reference's submodule names (embed, rnn, convs1, k, q), so their state dicts
load unchanged.  The word embedding, biGRU and Conv2d are frozen PyTorch backbones (the north
star leaves them to PyTorch-ROCm); the temporal pools -- per-caption mean over the valid steps
(model.py:238-241), masked max (:242-243) and the max_pool1d over the conv outputs (:247) -- run on
the K2 kernel, like the video side.

Vocabulary files: the reference pickles its Vocabulary objects (inference.py:69-74).  ``load_vocab``
reads JSON, or such a pickle through a restricted unpickler that admits only the Vocabulary class
and plain containers -- nothing in the file is executed.
"""
from __future__ import annotations

import io
import json
import pickle
import re
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.utils.rnn import pack_padded_sequence, pad_packed_sequence

from .model import temporal_pool


# ---------------------------------------------------------------- tokeniser / vocabularies
def clean_str(string: str) -> List[str]:
    """util/vocab.py:47-49."""
    string = re.sub(r"[^A-Za-z0-9]", " ", string)
    return string.strip().lower().split()


class Vocabulary:
    """util/vocab.py:15-35 (same attributes, so pickled reference vocabularies map onto it)."""

    def __init__(self, text_style: str):
        self.word2idx = {}
        self.idx2word = {}
        self.idx = 0
        self.text_style = text_style

    def add_word(self, word):
        if word not in self.word2idx:
            self.word2idx[word] = self.idx
            self.idx2word[self.idx] = word
            self.idx += 1

    def __call__(self, word):
        if word not in self.word2idx and 'bow' not in self.text_style:
            return self.word2idx['<unk>']
        return self.word2idx[word]

    def __len__(self):
        return len(self.word2idx)

    def to_json(self, path: str):
        with open(path, "w") as f:
            json.dump({"text_style": self.text_style, "words": [self.idx2word[i] for i in range(self.idx)]}, f)

    @classmethod
    def from_words(cls, words: Sequence[str], text_style: str) -> "Vocabulary":
        v = cls(text_style)
        for w in words:
            v.add_word(w)
        return v


def build_vocab(captions: Sequence[str], text_style: str, threshold: int = 4) -> Vocabulary:
    """util/vocab.py:60-88 over an in-memory caption list: words of clean_str(caption.lower()) seen at
    least `threshold` times, in first-occurrence order, after <pad> <start> <end> <unk> for 'rnn'."""
    from collections import Counter
    counter = Counter()
    for c in captions:
        counter.update(clean_str(c.lower()))
    vocab = Vocabulary(text_style)
    if 'rnn' in text_style:
        for w in ('<pad>', '<start>', '<end>', '<unk>'):
            vocab.add_word(w)
    for w, cnt in counter.items():
        if cnt >= threshold:
            vocab.add_word(w)
    return vocab


class _VocabUnpickler(pickle.Unpickler):
    """Admits the reference's Vocabulary class (any module path ending in 'vocab') and nothing else."""

    def find_class(self, module, name):
        if name == "Vocabulary" and module.split(".")[-1] == "vocab":
            return Vocabulary
        raise pickle.UnpicklingError(f"cmve.load_vocab: refusing to load {module}.{name} from a vocabulary file")


def load_vocab(path: str) -> Vocabulary:
    """A vocabulary from JSON (Vocabulary.to_json) or from the reference's pickle, restricted to the
    Vocabulary class and builtin containers."""
    with open(path, "rb") as f:
        data = f.read()
    if data.lstrip()[:1] == b"{":
        d = json.loads(data.decode("utf-8"))
        return Vocabulary.from_words(d["words"], d["text_style"])
    v = _VocabUnpickler(io.BytesIO(data)).load()
    if not isinstance(v, Vocabulary):
        raise pickle.UnpicklingError("cmve.load_vocab: the file does not hold a Vocabulary")
    return v


class Bow2Vec:
    """util/text2vec.py:49-74: bag-of-words counts over the vocabulary, optionally L1 / L2 normalised;
    None when no word of the query is in the vocabulary."""

    def __init__(self, vocab: Vocabulary, ndims: int = 0, L1_norm: int = 0, L2_norm: int = 0):
        assert (L1_norm + L2_norm) <= 1
        self.vocab = vocab
        self.L1_norm, self.L2_norm = L1_norm, L2_norm
        if ndims != 0:
            assert len(vocab) == ndims, "feature dimension not match %d != %d" % (len(vocab), ndims)
        self.ndims = len(vocab)

    def sparse(self, query: str, clear: bool = True):
        """mapping() as (columns, float64 values), or None: the same numbers without the dense
        ndims-long Python list (which dominated batched collation)."""
        words = clean_str(query) if clear else query.strip().split()
        counts = {}
        for word in words:
            if word in self.vocab.word2idx:
                j = self.vocab(word)
                counts[j] = counts.get(j, 0) + 1
        if not counts:
            return None
        cols = np.fromiter(counts.keys(), np.int64, len(counts))
        vals = np.fromiter(counts.values(), np.float64, len(counts))
        if self.L1_norm:
            vals = 1.0 * vals / np.abs(vals).sum()  # integer counts: every summation order is exact
        elif self.L2_norm:
            vals = 1.0 * vals / np.sqrt((vals * vals).sum())
        return cols, vals

    def mapping(self, query: str, clear: bool = True):
        words = clean_str(query) if clear else query.strip().split()
        vec = [0.0] * self.ndims
        for word in words:
            if word in self.vocab.word2idx:
                vec[self.vocab(word)] += 1
        if sum(vec) > 0:
            if self.L1_norm:
                return 1.0 * np.array(vec) / np.linalg.norm(vec, 1)
            if self.L2_norm:
                return 1.0 * np.array(vec) / np.linalg.norm(vec, 2)
            return np.array(vec)
        return None


def get_text_encoder(name: str):
    """util/text2vec.py:get_text_encoder for the 'bow' encoder (the one inference.py uses)."""
    if name == "bow":
        return Bow2Vec
    raise NotImplementedError(f"cmve: text encoder {name!r} is not on the MI355X path (bow only)")


def _caption_tensors(caption: str, vocab: Optional[Vocabulary], bow2vec: Optional[Bow2Vec]):
    """TxtDataSet4DualEncoding.process_cap (tag_data_provider.py:419-436) / inference.py:15-32."""
    cap_bow = None
    if bow2vec is not None:
        b = bow2vec.mapping(caption)
        cap_bow = torch.zeros(bow2vec.ndims) if b is None else torch.Tensor(b)
    cap_tensor = None
    if vocab is not None:
        tokens = clean_str(caption)
        ids = [vocab('<start>')] + [vocab(t) for t in tokens] + [vocab('<end>')]
        cap_tensor = torch.Tensor(ids)
    return cap_tensor, cap_bow


def process_cap(caption: str, vocab: Vocabulary, bow2vec: Bow2Vec):
    """inference.py:15-35: (word ids [1, L] long, bow [1, V], [L], mask ones [1, L])."""
    cap_tensor, cap_bow = _caption_tensors(caption, vocab, bow2vec)
    return (cap_tensor.long().unsqueeze(0), cap_bow.unsqueeze(0), [len(cap_tensor)],
            torch.ones(1, len(cap_tensor)))


def collate_text(captions: Sequence[str], vocab: Vocabulary, bow2vec: Optional[Bow2Vec], idxs=None, cap_ids=None,
                 device=None):
    """collate_text_distill (tag_data_provider.py:160-184) over raw captions: sorted by token length
    (descending, stable), zero-padded ids, float mask, stacked BoWs.  Returns
    ((target, cap_bows, lengths, words_mask), idxs, cap_ids) in the sorted order; with `device` the
    tensors are built there (BoWs scattered from their sparse counts)."""
    idxs = list(range(len(captions))) if idxs is None else list(idxs)
    cap_ids = list(idxs) if cap_ids is None else list(cap_ids)
    toks = [[vocab('<start>')] + [vocab(t) for t in clean_str(c)] + [vocab('<end>')] for c in captions]
    order = sorted(range(len(captions)), key=lambda k: len(toks[k]), reverse=True)  # stable, like list.sort
    lengths = [len(toks[k]) for k in order]
    B, L = len(order), max(lengths)
    target = np.zeros((B, L), np.int64)
    words_mask = np.zeros((B, L), np.float32)
    for r, k in enumerate(order):
        target[r, :lengths[r]] = toks[k]
        words_mask[r, :lengths[r]] = 1.0
    dev = torch.device(device) if device is not None else torch.device("cpu")
    cap_bows = None
    if bow2vec is not None:
        rows, cols, vals = [], [], []
        for r, k in enumerate(order):
            sp = bow2vec.sparse(captions[k])
            if sp is not None:
                rows.append(np.full(sp[0].size, r, np.int64))
                cols.append(sp[0])
                vals.append(sp[1].astype(np.float32))
        cap_bows = torch.zeros((B, bow2vec.ndims), dtype=torch.float32, device=dev)
        if rows:
            r_ = torch.from_numpy(np.concatenate(rows)).to(dev)
            c_ = torch.from_numpy(np.concatenate(cols)).to(dev)
            cap_bows[r_, c_] = torch.from_numpy(np.concatenate(vals)).to(dev)
    return ((torch.from_numpy(target).to(dev), cap_bows, lengths, torch.from_numpy(words_mask).to(dev)),
            tuple(idxs[k] for k in order), tuple(cap_ids[k] for k in order))


# ---------------------------------------------------------------- text encoders
def _gru_pool(gru_init_out: torch.Tensor, lengths, cap_mask, gru_pool: str) -> torch.Tensor:
    lens = torch.as_tensor(np.asarray([int(x) for x in lengths], np.int32))
    if gru_pool == 'mean':    # model.py:238-241: mean over the first lengths[i] steps
        return temporal_pool(gru_init_out.contiguous(), "mean_valid", lens)
    if gru_pool == 'max':     # model.py:242-243: max_t (x * mask) -- masked steps count as 0
        return temporal_pool(gru_init_out.contiguous(), "masked_max", lens)
    raise ValueError(f"gru_pool {gru_pool!r}")


def _conv_pool(gru_init_out: torch.Tensor, convs: nn.ModuleList) -> torch.Tensor:
    """Level 3 (model.py:245-248): relu(Conv2d) per window size, then max over the whole padded
    length (F.max_pool1d with the full width) on K2."""
    con_in = gru_init_out.unsqueeze(1)
    outs = [F.relu(conv(con_in)).squeeze(3) for conv in convs]                   # [B, C, T']
    outs = [temporal_pool(o.transpose(1, 2).contiguous(), "max") for o in outs]  # [B, C]
    return torch.cat(outs, 1)


class Text_multilevel_encoding_ori(nn.Module):
    """model.py:191-260 (eval forward; the frozen backbones stay PyTorch)."""

    def __init__(self, opt):
        super().__init__()
        self.word_dim = opt.word_dim
        self.we_parameter = getattr(opt, "we_parameter", None)
        self.rnn_output_size = opt.text_rnn_size * 2
        self.dropout = nn.Dropout(p=opt.dropout)
        self.concate = opt.concate
        self.gru_pool = opt.gru_pool
        self.loss_fun = getattr(opt, "loss_fun", "mrl")
        self.embed = nn.Embedding(opt.vocab_size, opt.word_dim)
        self.rnn = nn.GRU(opt.word_dim, opt.text_rnn_size, batch_first=True, bidirectional=True)
        self.convs1 = nn.ModuleList([
            nn.Conv2d(1, opt.text_kernel_num, (w, self.rnn_output_size), padding=(w - 1, 0))
            for w in opt.text_kernel_sizes])
        if self.word_dim == 500 and self.we_parameter is not None:
            self.embed.weight.data.copy_(torch.from_numpy(self.we_parameter))
        else:
            self.embed.weight.data.uniform_(-0.1, 0.1)

    def _check_eval(self):
        if self.training:
            raise NotImplementedError("cmve text encoders are the frozen query-side backbones: call .eval()")

    def encode_text(self, cap_wids, cap_bows, lengths, cap_mask, sort=False):
        lengths_l = [int(x) for x in (lengths.tolist() if torch.is_tensor(lengths) else lengths)]
        emb = self.embed(cap_wids)
        if sort:  # model.py:323-331: torch.sort by length, pack, unpack, restore the order
            sorted_len, indices = torch.sort(torch.as_tensor(lengths_l), descending=True)
            _, desorted = torch.sort(indices, descending=False)
            dev = emb.device
            packed = pack_padded_sequence(emb[indices.to(dev)], sorted_len.numpy(), batch_first=True)
            out, _ = self.rnn(packed)
            padded, _ = pad_packed_sequence(out, batch_first=True)
            gru_init_out = padded[desorted.to(dev)]
            # model.py:335-337 averages the rows of the SORTED `padded` over the UNSORTED lengths (and
            # leaves the result in sorted order); reproduced, not fixed
            mean_src = padded
        else:     # model.py:229-234: the caller sorted the batch (collate_text)
            packed = pack_padded_sequence(emb, lengths_l, batch_first=True)
            out, _ = self.rnn(packed)
            gru_init_out = pad_packed_sequence(out, batch_first=True)[0]
            mean_src = gru_init_out
        gru_out = _gru_pool(mean_src if self.gru_pool == 'mean' else gru_init_out, lengths_l, cap_mask, self.gru_pool)
        con_out = _conv_pool(gru_init_out, self.convs1)
        if self.concate == 'full':
            return torch.cat((gru_out, con_out, cap_bows.to(gru_out.dtype)), 1)
        return torch.cat((gru_out, con_out), 1)

    def forward(self, text, *args):
        self._check_eval()
        cap_wids, cap_bows, lengths, cap_mask = text
        return self.encode_text(cap_wids, cap_bows, lengths, cap_mask, sort=False)


class Text_multilevel_encoding(Text_multilevel_encoding_ori):
    """model.py:263-359: encode_text sorts internally; with a support set, the support captions are
    gated by softmax(k(s_feature) . q(feature)) and added ('GT') or returned beside ('distill')."""

    def __init__(self, opt):
        super().__init__(opt)
        self.style = opt.style
        self.teacher_model = getattr(opt, "teacher_model", None)
        self.k = nn.Linear(opt.text_mapping_layers[0], opt.hidden_size, bias=True)
        self.q = nn.Linear(opt.text_mapping_layers[0], opt.hidden_size, bias=True)

    def forward(self, text, support_text=None, *args):
        self._check_eval()
        cap_wids, cap_bows, lengths, cap_mask = text
        feature = self.encode_text(cap_wids, cap_bows, lengths, cap_mask, sort=True)
        if support_text is None:
            return feature
        s_wids, s_bows, s_lengths, s_mask = support_text
        s_lengths = torch.as_tensor(np.asarray(s_lengths))
        s_feature = torch.stack([self.encode_text(s_wids[:, i, :], s_bows[:, i, :], s_lengths[:, i], s_mask[:, i, :],
                                                  sort=True) for i in range(s_wids.size(1))], 1)
        key = self.k(s_feature)
        query = self.q(feature)
        w = F.softmax(torch.bmm(key, query.unsqueeze(2)), dim=1)
        w = w.repeat(1, 1, s_feature.shape[2])
        gated = torch.sum(w * s_feature, dim=1)
        if self.style == 'distill_from_best_model':
            return feature, gated
        if self.style == 'GT':
            return feature + gated
        return None
