"""Golden vectors for the query-side row, produced by running the REFERENCE's
own code in the build container:

  LINAS-engine/util/vocab.py:15-88          Vocabulary, clean_str, build_vocab (rnn + bow styles)
  LINAS-engine/util/text2vec.py:49-74,120    Bow2Vec via get_text_encoder('bow') (plain, L1, L2)
  LINAS-engine/inference.py:15-35            process_cap (module globals vocab / bow2vec set here)
  LINAS-engine/util/tag_data_provider.py:160 collate_text_distill
  LINAS-engine/model.py:191-359              Text_multilevel_encoding_ori (gru_pool mean / max,
                                             concate full / reduced) and Text_multilevel_encoding
                                             (+ support set, style GT), eval mode, seeded weights

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_text.py /root/reference
Writes tests/golden/text.npz, plus text_rnn_vocab.pkl / text_bow_vocab.pkl: the reference's
Vocabulary objects pickled by the reference's own pickle.dump (build_vocab's main, vocab.py:106-108),
to test the restricted loader.  torch.Tensor.cuda is patched to identity (model.py:239).
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

CAPTIONS = [
    "A man and a woman is talking.", "a dog runs on the grass", "Two men are playing guitar!!",
    "a woman is cooking in a kitchen", "the man rides a bike down the street", "a cat sits on a table",
    "people are dancing at a party", "A man is talking about cars", "a girl is singing a song",
    "a dog and a cat play", "someone slices an onion", "the woman talks to the man",
]
QUERIES = ["a man and a woman is talking.", "zebra quantum", "A DOG plays; with a cat...", "man man man"]


def text_opt(vocab_size, bow_dim, gru_pool, concate, style="GT"):
    rnn_out, kn, ks = 2 * 8, 4, [2, 3, 4]
    in_dim = rnn_out + kn * len(ks) + (bow_dim if concate == "full" else 0)
    return argparse.Namespace(word_dim=16, we_parameter=None, text_rnn_size=8, dropout=0.2, concate=concate,
                              gru_pool=gru_pool, loss_fun="mrl", vocab_size=vocab_size, text_kernel_num=kn,
                              text_kernel_sizes=ks, style=style, teacher_model="teacher",
                              text_mapping_layers=[in_dim, 32], hidden_size=10)


def main(ref_root):
    sys.path.insert(0, os.path.join(ref_root, "LINAS-engine"))
    torch.Tensor.cuda = lambda self, *a, **k: self
    from util import vocab as V  # noqa
    from util import text2vec as T2V  # noqa
    from util import tag_data_provider as TDP  # noqa
    import inference as INF  # noqa  (script body is under __main__)
    import model as M  # noqa

    out = {}
    with tempfile.TemporaryDirectory() as d:
        cap_file = os.path.join(d, "caps.txt")
        with open(cap_file, "w") as f:
            for i, c in enumerate(CAPTIONS):
                f.write(f"vid{i}#0 {c}\n")
        rnn_vocab, _ = V.build_vocab(cap_file, "rnn", threshold=1)
        bow_vocab, _ = V.build_vocab(cap_file, "bow", threshold=2)
    with open(os.path.join(HERE, "text_rnn_vocab.pkl"), "wb") as f:
        pickle.dump(rnn_vocab, f, pickle.HIGHEST_PROTOCOL)
    with open(os.path.join(HERE, "text_bow_vocab.pkl"), "wb") as f:
        pickle.dump(bow_vocab, f, pickle.HIGHEST_PROTOCOL)
    out["rnn_words"] = np.array([rnn_vocab.idx2word[i] for i in range(len(rnn_vocab))])
    out["bow_words"] = np.array([bow_vocab.idx2word[i] for i in range(len(bow_vocab))])
    for q, s in enumerate(CAPTIONS + QUERIES):
        out[f"clean{q}"] = np.array(V.clean_str(s) or [""])
    for name, kw in (("plain", {}), ("l1", {"L1_norm": 1}), ("l2", {"L2_norm": 1})):
        b2v = T2V.get_text_encoder("bow")(bow_vocab, **kw)
        for q, s in enumerate(QUERIES):
            v = b2v.mapping(s)
            out[f"bow_{name}_{q}"] = np.zeros(0) if v is None else np.asarray(v, np.float64)
    INF.vocab = rnn_vocab
    INF.bow2vec = T2V.get_text_encoder("bow")(bow_vocab)
    for q, s in enumerate(QUERIES):
        ids, bow, lens, mask = INF.process_cap(s)
        out[f"pc{q}_ids"], out[f"pc{q}_bow"] = ids.numpy(), bow.numpy()
        out[f"pc{q}_len"], out[f"pc{q}_mask"] = np.array(lens), mask.numpy()

    # collate_text_distill over dataset-style items (TxtDataSet4DualEncoding.process_cap, :419-436)
    items = []
    for i, c in enumerate(CAPTIONS):
        bow = INF.bow2vec.mapping(c)
        bow = torch.zeros(INF.bow2vec.ndims) if bow is None else torch.Tensor(bow)
        ids = torch.Tensor([rnn_vocab('<start>')] + [rnn_vocab(t) for t in V.clean_str(c)] + [rnn_vocab('<end>')])
        items.append((ids, bow, i, f"vid{i}#0"))
    (target, bows, lengths, mask), idxs, cap_ids = TDP.collate_text_distill(items)
    out.update(col_target=target.numpy(), col_bows=bows.numpy(), col_lengths=np.array(lengths),
               col_mask=mask.numpy(), col_idxs=np.array(idxs))

    # text encoders (eval), batch = the collated captions
    lengths_t = torch.Tensor(lengths)  # embed_txt_distill (model.py:765-767)
    for pool in ("mean", "max"):
        for concate in ("full", "reduced"):
            torch.manual_seed(31)
            enc = M.Text_multilevel_encoding_ori(text_opt(len(rnn_vocab), INF.bow2vec.ndims, pool, concate)).eval()
            with torch.no_grad():
                feats = enc((target, bows, lengths_t, mask))
            key = f"ori_{pool}_{concate}"
            out[key] = feats.numpy()
            out.update({f"{key}.sd.{k}": v.numpy() for k, v in enc.state_dict().items()})
    # support-set encoder, style GT: 3 support captions per query
    torch.manual_seed(37)
    opt = text_opt(len(rnn_vocab), INF.bow2vec.ndims, "mean", "full")
    enc = M.Text_multilevel_encoding(opt).eval()
    B, S = 5, 3
    g = torch.Generator().manual_seed(3)
    s_len = torch.randint(3, 9, (B, S), generator=g)
    m = int(s_len.max())
    s_ids = torch.zeros(B, S, m).long()
    s_mask = torch.zeros(B, S, m)
    for b in range(B):
        for s in range(S):
            s_ids[b, s, :s_len[b, s]] = torch.randint(1, len(rnn_vocab), (int(s_len[b, s]),), generator=g)
            s_mask[b, s, :s_len[b, s]] = 1.0
    s_bows = torch.rand(B, S, INF.bow2vec.ndims, generator=g)
    q_ids, q_bows, q_len, q_mask = target[:B], bows[:B], lengths_t[:B], mask[:B]
    with torch.no_grad():
        feats = enc((q_ids, q_bows, q_len, q_mask), (s_ids, s_bows, s_len.float(), s_mask))
        plain = enc((q_ids, q_bows, q_len, q_mask), None)
    out.update(sup_s_ids=s_ids.numpy(), sup_s_bows=s_bows.numpy(), sup_s_len=s_len.numpy(), sup_s_mask=s_mask.numpy(),
               sup_feats=feats.numpy(), sup_plain=plain.numpy())
    out.update({f"sup.sd.{k}": v.numpy() for k, v in enc.state_dict().items()})
    np.savez_compressed(os.path.join(HERE, "text.npz"), **out)
    print(len(out), "arrays;", len(rnn_vocab), "rnn words;", len(bow_vocab), "bow words")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
