"""Query-side row: tokeniser, vocabularies, BoW, process_cap, caption collation
(host logic, CPU) and the text encoders with the pools on the HIP kernels (GPU), against
tests/golden/text.npz from the reference's own code (tests/golden/make_golden_text.py).
"""
import os
import pickle

import numpy as np
import pytest
import torch

from oracle import text as OT

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
CAPTIONS = ["A man and a woman is talking.", "a dog runs on the grass", "Two men are playing guitar!!",
            "a woman is cooking in a kitchen", "the man rides a bike down the street", "a cat sits on a table",
            "people are dancing at a party", "A man is talking about cars", "a girl is singing a song",
            "a dog and a cat play", "someone slices an onion", "the woman talks to the man"]  # = make_golden_text
QUERIES = ["a man and a woman is talking.", "zebra quantum", "A DOG plays; with a cat...", "man man man"]
KS, H = [2, 3, 4], 8


def _vocabs():
    from cmve.linas import text as T
    return T.load_vocab(os.path.join(GOLD, "text_rnn_vocab.pkl")), T.load_vocab(os.path.join(GOLD, "text_bow_vocab.pkl"))


def test_host_text_pipeline_matches_reference(golden):
    from cmve.linas import text as T
    g = golden("text")
    rnn, bow = _vocabs()
    assert [rnn.idx2word[i] for i in range(len(rnn))] == list(g["rnn_words"])
    assert [bow.idx2word[i] for i in range(len(bow))] == list(g["bow_words"])
    assert [w for w in T.build_vocab(CAPTIONS, "rnn", 1).word2idx] == list(g["rnn_words"])
    assert [w for w in T.build_vocab(CAPTIONS, "bow", 2).word2idx] == list(g["bow_words"])
    for q, s in enumerate(CAPTIONS + QUERIES):
        assert (T.clean_str(s) or [""]) == list(g[f"clean{q}"])
    for name, kw in (("plain", {}), ("l1", {"L1_norm": 1}), ("l2", {"L2_norm": 1})):
        b2v = T.get_text_encoder("bow")(bow, **kw)
        for q, s in enumerate(QUERIES):
            v = b2v.mapping(s)
            want = g[f"bow_{name}_{q}"]
            if want.size == 0:
                assert v is None
            else:
                np.testing.assert_array_equal(v, want)
    b2v = T.Bow2Vec(bow)
    for q, s in enumerate(QUERIES):
        ids, bw, lens, mask = T.process_cap(s, rnn, b2v)
        np.testing.assert_array_equal(ids.numpy(), g[f"pc{q}_ids"])
        np.testing.assert_array_equal(bw.numpy(), g[f"pc{q}_bow"])
        assert lens == list(g[f"pc{q}_len"])
        np.testing.assert_array_equal(mask.numpy(), g[f"pc{q}_mask"])
    for kw in ({}, {"L1_norm": 1}, {"L2_norm": 1}):  # sparse == dense mapping, bit for bit
        bb = T.Bow2Vec(bow, **kw)
        for s in CAPTIONS + QUERIES:
            dense, sp = bb.mapping(s), bb.sparse(s)
            if dense is None:
                assert sp is None
            else:
                v = np.zeros(bb.ndims)
                v[sp[0]] = sp[1]
                np.testing.assert_array_equal(v, dense)
    (target, bows, lengths, mask), idxs, _ = T.collate_text(CAPTIONS, rnn, b2v)
    np.testing.assert_array_equal(target.numpy(), g["col_target"])
    np.testing.assert_array_equal(bows.numpy(), g["col_bows"])
    assert lengths == list(g["col_lengths"])
    np.testing.assert_array_equal(mask.numpy(), g["col_mask"])
    assert list(idxs) == list(g["col_idxs"])


def test_vocab_loader_is_restricted(tmp_path):
    from cmve.linas import text as T
    rnn, _ = _vocabs()
    rnn.to_json(str(tmp_path / "v.json"))
    again = T.load_vocab(str(tmp_path / "v.json"))
    assert again.word2idx == rnn.word2idx and again.text_style == rnn.text_style

    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    (tmp_path / "evil.pkl").write_bytes(pickle.dumps(Evil()))
    with pytest.raises(pickle.UnpicklingError, match="refusing"):
        T.load_vocab(str(tmp_path / "evil.pkl"))


def test_oracle_text_encoders_match_reference(golden):
    g = golden("text")
    ids, bows, lengths = g["col_target"], g["col_bows"], g["col_lengths"]
    for pool in ("mean", "max"):
        for concate in ("full", "reduced"):
            key = f"ori_{pool}_{concate}"
            sd = {k[len(key) + 4:]: g[k] for k in g.files if k.startswith(key + ".sd.")}
            got = OT.encode_text(sd, "", ids, bows, lengths, KS, H, pool, concate)
            np.testing.assert_allclose(got, g[key], rtol=1e-5, atol=1e-6, err_msg=key)
    sd = {k[7:]: g[k] for k in g.files if k.startswith("sup.sd.")}
    B, S = 5, 3
    f = OT.encode_text(sd, "", ids[:B], bows[:B], lengths[:B], KS, H, "mean", "full", sorted_mean=True)
    np.testing.assert_allclose(f, g["sup_plain"], rtol=1e-5, atol=1e-6)
    sf = np.stack([OT.encode_text(sd, "", g["sup_s_ids"][:, s], g["sup_s_bows"][:, s], g["sup_s_len"][:, s], KS, H,
                                  "mean", "full", sorted_mean=True) for s in range(S)], 1)
    np.testing.assert_allclose(f + OT.support_gate(sd, "", f, sf), g["sup_feats"], rtol=1e-5, atol=1e-6)


def _opt(vocab_size, bow_dim, pool, concate, style="GT"):
    import argparse
    in_dim = 2 * H + 4 * len(KS) + (bow_dim if concate == "full" else 0)
    return argparse.Namespace(word_dim=16, we_parameter=None, text_rnn_size=H, dropout=0.2, concate=concate,
                              gru_pool=pool, loss_fun="mrl", vocab_size=vocab_size, text_kernel_num=4,
                              text_kernel_sizes=KS, style=style, teacher_model="teacher",
                              text_mapping_layers=[in_dim, 32], hidden_size=10)


@pytest.mark.gpu
def test_text_encoders_match_reference(golden):
    from cmve.linas import text as T
    g = golden("text")
    rnn, bow = _vocabs()
    dev = torch.device("cuda")
    ids = torch.from_numpy(g["col_target"]).to(dev)
    bows = torch.from_numpy(g["col_bows"]).to(dev)
    mask = torch.from_numpy(g["col_mask"]).to(dev)
    lengths = torch.Tensor(g["col_lengths"].astype(np.float32))
    for pool in ("mean", "max"):
        for concate in ("full", "reduced"):
            key = f"ori_{pool}_{concate}"
            enc = T.Text_multilevel_encoding_ori(_opt(len(rnn), len(bow), pool, concate)).to(dev).eval()
            enc.load_state_dict({k[len(key) + 4:]: torch.from_numpy(g[k]) for k in g.files if k.startswith(key + ".sd.")})
            with torch.no_grad():
                got = enc((ids, bows, lengths, mask))
            np.testing.assert_allclose(got.cpu().numpy(), g[key], rtol=1e-5, atol=1e-6, err_msg=key)
    enc = T.Text_multilevel_encoding(_opt(len(rnn), len(bow), "mean", "full")).to(dev).eval()
    enc.load_state_dict({k[7:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("sup.sd.")})
    B = 5
    q = (ids[:B], bows[:B], lengths[:B], mask[:B])
    s = (torch.from_numpy(g["sup_s_ids"]).to(dev), torch.from_numpy(g["sup_s_bows"]).to(dev),
         torch.from_numpy(g["sup_s_len"]).float(), torch.from_numpy(g["sup_s_mask"]).to(dev))
    with torch.no_grad():
        np.testing.assert_allclose(enc(q, None).cpu().numpy(), g["sup_plain"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(enc(q, s).cpu().numpy(), g["sup_feats"], rtol=1e-5, atol=1e-6)
    with pytest.raises(NotImplementedError, match="eval"):
        enc.train()(q, None)


def _fake_checkpoint(path, rnn, bow, student_model="de+map"):
    """A checkpoint in the reference's layout (trainer.py:288-293), with a numpy array in opt."""
    from cmve.linas import text as T
    from cmve.linas.model import Latent_mapping
    opt = _opt(len(rnn), len(bow), "mean", "full")
    opt.student_model, opt.dropout, opt.tag_vocab_size = student_model, 0.2, 512
    opt.we_parameter = np.zeros((3, 2), np.float32)  # the reference stores the word2vec matrix in opt
    torch.manual_seed(5)
    enc = T.Text_multilevel_encoding_ori(opt)
    mapping = Latent_mapping(opt.text_mapping_layers, 0.2)
    slots = [None] * 9
    slots[4], slots[5] = mapping.state_dict(), enc.state_dict()
    torch.save({"epoch": 3, "model": slots, "best_rsum": 1.0, "opt": opt, "Eiters": 7}, path)
    return opt, enc, mapping


def test_checkpoint_loads_weights_only_and_refuses_code(tmp_path):
    from cmve.linas.checkpoint import load_checkpoint
    rnn, bow = _vocabs()
    _fake_checkpoint(str(tmp_path / "ck.pth.tar"), rnn, bow)
    ck = load_checkpoint(str(tmp_path / "ck.pth.tar"))
    assert ck["Eiters"] == 7 and ck["opt"].student_model == "de+map" and ck["opt"].we_parameter.shape == (3, 2)

    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    torch.save({"opt": Evil()}, str(tmp_path / "evil.pth.tar"))
    with pytest.raises(Exception, match="(?i)weights.only|unsupported|global"):
        load_checkpoint(str(tmp_path / "evil.pth.tar"))


@pytest.mark.gpu
def test_query_encoder_from_checkpoint(tmp_path):
    """QueryEncoder == student_text_mapping(student_text_encoding(process_cap(...))) composed by hand,
    and batched encode_captions (collate sorts) restores the input order."""
    from cmve.linas import text as T
    from cmve.linas.checkpoint import QueryEncoder
    rnn, bow = _vocabs()
    _, enc, mapping = _fake_checkpoint(str(tmp_path / "ck.pth.tar"), rnn, bow)
    qe = QueryEncoder.from_checkpoint(str(tmp_path / "ck.pth.tar"))
    b2v = T.Bow2Vec(bow)
    enc = enc.cuda().eval()
    mapping = mapping.cuda().eval()
    one = []
    for q in QUERIES:
        txt = T.process_cap(q, rnn, b2v)
        got = qe(txt)
        ids, bw, lens, mask = txt
        want = mapping(enc((ids.cuda(), bw.cuda(), torch.Tensor(lens), mask.cuda())))
        torch.testing.assert_close(got, want, rtol=0, atol=0)
        one.append(got[0].cpu().numpy())
    # batched: the conv max runs over the batch's padded width (model.py:247), so a
    # caption's embedding depends on its batch exactly as in the reference's encode_text
    batch = qe.encode_captions(QUERIES, rnn, b2v, batch_size=len(QUERIES))
    (ids, bw, lens, mask), idxs, _ = T.collate_text(QUERIES, rnn, b2v)
    want = mapping(enc((ids.cuda(), bw.cuda(), torch.Tensor(lens), mask.cuda()))).cpu().numpy()
    np.testing.assert_allclose(batch[list(idxs)], want, rtol=0, atol=0)
    np.testing.assert_allclose(batch[0], one[0], rtol=1e-5, atol=1e-6)  # the longest caption sees no extra padding
