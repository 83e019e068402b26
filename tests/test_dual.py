"""Video-side encoder facade, encode_vid and the inference.py drop-in CLI.

Golden: tests/golden/dual_{tv,dm}.{pth.tar,npz}, made by tests/golden/make_golden_dual.py running
the reference's Dual_Encoding (student 'text+video' with gru_pool max, 'de+map' with gru_pool mean)
over the toy BigFile gallery: its 9-slot checkpoint, encode_vid(embed_vis_distill / embed_vis)
output, embed_txt_distill(process_cap(q)) and inference.py's printed top-10 id list.
Tolerances: embeddings atol 1e-5 on unit-norm rows (the fp32 biGRU recurrence on MIOpen vs the
reference's CPU ATen run differs by ~3e-6; split-bf16 heads ~1e-6), inside the north-star 1e-4;
id lists exact.
"""
import os
import shutil

import numpy as np
import pytest
import torch

import make_golden_dual as MG
import synth

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MODELS = ["tv", "dm"]


def _ck(name):
    return os.path.join(GOLD, f"dual_{name}.pth.tar")


@pytest.mark.parametrize("name", MODELS)
def test_dual_slots_round_trip_on_cpu(name):
    """get_model(opt.model)(opt).load_state_dict(slots, 'test') fills the reference's modules:
    state_dict() returns the checkpoint's slots key for key, tensor for tensor."""
    from cmve.linas.checkpoint import get_model, load_checkpoint
    ck = load_checkpoint(_ck(name))
    model = get_model(ck["opt"].model)(ck["opt"], device=torch.device("cpu"))
    model.load_state_dict(ck["model"], "test")
    got = model.state_dict()
    for slot, (a, b) in enumerate(zip(got, ck["model"])):
        assert (a is None) == (b is None), slot
        if a is None:
            continue
        assert list(a.keys()) == list(b.keys()), slot
        for k in a:
            assert torch.equal(a[k], b[k]), (slot, k)
    with pytest.raises(AssertionError):
        get_model("nope")


def _toy_loader(tmp, batch, device=None):
    from cmve.linas.bigfile import BigFile, VideoBatchLoader, read_dict
    synth.bigfile_toy(tmp, dim=MG.FEAT)
    v2f = read_dict(os.path.join(tmp, "video2frames.txt"))
    return VideoBatchLoader(BigFile(tmp), v2f, video_ids=list(v2f.keys()), batch_size=batch, device=device)


@pytest.mark.gpu
@pytest.mark.parametrize("name", MODELS)
def test_encode_vid_matches_reference(name, tmp_path):
    from cmve.linas.checkpoint import Dual_Encoding
    from cmve.linas.evaluation import encode_vid
    g = np.load(os.path.join(GOLD, f"dual_{name}.npz"))
    model = Dual_Encoding.from_checkpoint(_ck(name))
    loader = _toy_loader(str(tmp_path), MG.BATCH)
    embs, ids = encode_vid(model.embed_vis_distill, loader)
    assert ids == list(g["video_ids"])
    assert embs.dtype == np.float64 and embs.shape == g["video_embs"].shape
    np.testing.assert_allclose(embs, g["video_embs"], rtol=1e-5, atol=1e-5)
    teacher = encode_vid(model.embed_vis, loader, return_ids=False)
    np.testing.assert_allclose(teacher, g["video_embs_teacher"], rtol=1e-5, atol=1e-5)
    for q, s in enumerate(MG.QUERIES):
        from cmve.linas import text as T
        rnn = T.load_vocab(os.path.join(GOLD, "text_rnn_vocab.pkl"))
        b2v = T.get_text_encoder("bow")(T.load_vocab(os.path.join(GOLD, "text_bow_vocab.pkl")))
        cap = model.embed_txt_distill(T.process_cap(s, rnn, b2v)).cpu().numpy()
        np.testing.assert_allclose(cap, g[f"q{q}_cap_emb"], rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_video_encoder_rejects_train_mode():
    from cmve.linas.checkpoint import load_checkpoint
    from cmve.linas.model import Video_multilevel_encoding
    enc = Video_multilevel_encoding(load_checkpoint(_ck("tv"))["opt"]).cuda()
    with pytest.raises(NotImplementedError, match="eval"):
        enc((torch.zeros(1, 2, MG.FEAT).cuda(), torch.zeros(1, MG.FEAT).cuda(), [2], torch.ones(1, 2).cuda()))


def _reference_layout(root, name):
    """The directory inference.py runs in: student_support_set_8/model_best.pth.tar and dataset/."""
    from cmve.linas.checkpoint import load_checkpoint
    opt = load_checkpoint(_ck(name))["opt"]
    os.makedirs(os.path.join(root, "student_support_set_8"))
    shutil.copy(_ck(name), os.path.join(root, "student_support_set_8", "model_best.pth.tar"))
    feat = os.path.join(root, "dataset", opt.collections_pathname["test"], "FeatureData", opt.visual_feature)
    synth.bigfile_toy(feat, dim=MG.FEAT)
    voc = os.path.join(root, "dataset", opt.collections_pathname["train"], "TextData", "vocabulary")
    for style in ("rnn", "bow"):
        os.makedirs(os.path.join(voc, style))
        shutil.copy(os.path.join(GOLD, f"text_{style}_vocab.pkl"), os.path.join(voc, style, opt.vocab + ".pkl"))


@pytest.mark.gpu
@pytest.mark.parametrize("name", MODELS)
def test_inference_cli_prints_reference_ids(name, tmp_path, monkeypatch, capsys):
    """python -m cmve.linas.inference in the reference's layout: the first run encodes the BigFile
    gallery and writes video_data.pt, the second reads it back; both print inference.py's list."""
    from cmve.linas import inference as INF
    from cmve.linas.bigfile import load_video_cache
    g = np.load(os.path.join(GOLD, f"dual_{name}.npz"))
    _reference_layout(str(tmp_path), name)
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", os.environ.get("HIP_VISIBLE_DEVICES", "0"))
    for q, s in enumerate(MG.QUERIES):
        want = [str(v) for v in g[f"q{q}_results"]]
        got = INF.main(["--input", s, "--topK", str(MG.TOPK), "--gpu", "0"])
        assert got == want, (q, s)
        assert capsys.readouterr().out.strip().splitlines()[-1] == str(want)  # after BigFile's load line
        if q == 0:
            embs, ids = load_video_cache("video_data.pt")
            assert ids == list(g["video_ids"])
            np.testing.assert_allclose(embs, g["video_embs"], rtol=1e-5, atol=1e-5)
