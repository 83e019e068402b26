"""CPU oracle for the query-side row.

TEST INFRASTRUCTURE ONLY (see oracle/retrieval.py).  A restatement of the reference text encoders'
forward (LINAS-engine/model.py:191-359): torch CPU for the word embedding / biGRU / Conv2d (the
frozen backbones) and numpy fp64 for everything the MI355X path does itself (the mean / masked-max
pools, the max over the conv outputs, the concatenation, the support-set gate).  Pinned against
tests/golden/text.npz, produced by the reference's own modules (tests/golden/make_golden_text.py).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F
from torch.nn.utils.rnn import pack_padded_sequence, pad_packed_sequence


def _backbone(sd, prefix, ids, lengths, kernel_sizes, hidden):
    """embed -> biGRU (packed via torch.sort order, model.py:323-331) -> (padded [B, T, 2H] in input
    order, the same rows in sorted order, the relu'd conv maps)."""
    word_dim = sd[prefix + "embed.weight"].shape[1]
    emb = F.embedding(torch.as_tensor(ids).long(), torch.as_tensor(sd[prefix + "embed.weight"]))
    rnn = torch.nn.GRU(word_dim, hidden, batch_first=True, bidirectional=True)
    rnn.load_state_dict({k[len(prefix) + 4:]: torch.as_tensor(v) for k, v in sd.items() if k.startswith(prefix + "rnn.")})
    lengths = [int(x) for x in lengths]
    sorted_len, order = torch.sort(torch.as_tensor(lengths), descending=True)
    _, inv = torch.sort(order, descending=False)
    with torch.no_grad():
        out, _ = rnn(pack_padded_sequence(emb[order], sorted_len.numpy(), batch_first=True))
        padded = pad_packed_sequence(out, batch_first=True)[0]
        gru = padded[inv]
        convs = []
        for k, w in enumerate(kernel_sizes):
            cw = torch.as_tensor(sd[f"{prefix}convs1.{k}.weight"])
            cb = torch.as_tensor(sd[f"{prefix}convs1.{k}.bias"])
            convs.append(F.relu(F.conv2d(gru.unsqueeze(1), cw, cb, padding=(w - 1, 0))).squeeze(3).numpy())
    return gru.numpy().astype(np.float64), padded.numpy().astype(np.float64), convs


def encode_text(sd, prefix, ids, bows, lengths, kernel_sizes, hidden, gru_pool, concate, sorted_mean=False):
    """sorted_mean: Text_multilevel_encoding.encode_text's mean pool (model.py:335-337), which averages
    the rows of the sorted `padded` over the unsorted lengths; the _ori encoder (model.py:238-241)
    gets a presorted batch, where both coincide."""
    gru, padded, convs = _backbone(sd, prefix, ids, lengths, kernel_sizes, hidden)
    lengths = [int(x) for x in lengths]
    if gru_pool == "mean":
        src = padded if sorted_mean else gru
        g = np.stack([src[i, :lengths[i]].mean(0) for i in range(len(lengths))])
    else:                    # model.py:242-243: masked steps count as 0
        mask = (np.arange(gru.shape[1])[None, :] < np.asarray(lengths)[:, None]).astype(np.float64)
        g = (gru * mask[:, :, None]).max(1)
    c = np.concatenate([x.astype(np.float64).max(2) for x in convs], 1)   # max_pool1d over the full width
    if concate == "full":
        return np.concatenate([g, c, np.asarray(bows, np.float64)], 1)
    return np.concatenate([g, c], 1)


def support_gate(sd, prefix, feature, s_feature):
    """model.py:312-318: softmax(k(s) . q(f)) over the support axis, weighted sum."""
    key = s_feature @ sd[prefix + "k.weight"].T.astype(np.float64) + sd[prefix + "k.bias"]
    query = feature @ sd[prefix + "q.weight"].T.astype(np.float64) + sd[prefix + "q.bias"]
    logits = np.einsum("bsh,bh->bs", key, query)
    w = np.exp(logits - logits.max(1, keepdims=True))
    w /= w.sum(1, keepdims=True)
    return (w[:, :, None] * s_feature).sum(1)
