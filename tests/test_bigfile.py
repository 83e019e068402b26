"""On-disk feature store row: BigFile / read_dict / video batch loader.

CPU tests: the oracle restatement and the native reader (libcmve host code, no GPU needed)
against tests/golden/bigfile.npz, produced by the reference's own basic/bigfile.py,
basic/util.py and util/tag_data_provider.py (tests/golden/make_golden_bigfile.py).
GPU tests: the HBM gather and the collate-on-device loader against the same vectors.
"""
import os

import numpy as np
import pytest

import synth
from oracle import bigfile as OB

BATCHES = [list(range(0, 16)), [1, 0, 7, 39, 12]]  # = make_golden_bigfile.BATCHES


@pytest.fixture(scope="module")
def toy(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("bigfile"))
    names, feats, v2f = synth.bigfile_toy(d)
    return d, names, feats, v2f


def _check_reads(bf, g):
    for q, req in enumerate(synth.BIGFILE_REQUESTS):
        names, vecs = bf.read(req)
        assert list(names) == list(g[f"read{q}_names"])
        assert np.array_equal(np.asarray(vecs, np.float32), g[f"read{q}_vecs"])
    names, vecs = bf.read([5, 2, 2, 0, 17], isname=False)
    assert list(names) == list(g["readidx_names"])
    assert np.array_equal(np.asarray(vecs, np.float32), g["readidx_vecs"])
    assert np.array_equal(np.asarray(bf.read_one("vid002_1"), np.float32), g["read_one"])
    assert bf.read(["nope"]) == ([], [])


def test_oracle_matches_reference_golden(toy, golden):
    d, _, _, _ = toy
    g = golden("bigfile")
    _check_reads(OB.BigFileOracle(d), g)
    v2f = OB.read_dict(os.path.join(d, "video2frames.txt"))
    vids = sorted(v2f)
    assert vids == list(g["video_ids"])
    bf = OB.BigFileOracle(d)
    for b, sel in enumerate(BATCHES):
        fl = []
        for i in sel:
            names, vecs = bf.read(v2f[vids[i]])
            order = {n: k for k, n in enumerate(names)}
            fl.append([vecs[order[f]] for f in v2f[vids[i]]])  # frame order of video2frames
        videos, origin, lengths, mask = OB.collate(fl)
        assert np.array_equal(videos, g[f"batch{b}_videos"])
        assert lengths == list(g[f"batch{b}_lengths"])
        assert np.array_equal(mask, g[f"batch{b}_mask"])
        np.testing.assert_allclose(origin, g[f"batch{b}_origin"], rtol=0, atol=2e-6)  # torch vs numpy mean


def test_native_reader_matches_reference_golden(toy, golden):
    from cmve.linas.bigfile import BigFile, read_dict
    d, names, feats, v2f = toy
    g = golden("bigfile")
    bf = BigFile(d)
    assert bf.shape() == [len(names), feats.shape[1]]
    _check_reads(bf, g)
    assert read_dict(os.path.join(d, "video2frames.txt")) == v2f
    rows = np.array([0, len(names) - 1, 3, 3, 17], np.int64)
    assert np.array_equal(bf.read_rows(rows), feats[rows])
    big = np.random.default_rng(0).integers(0, len(names), 20000)  # multi-threaded gather
    assert np.array_equal(bf.read_rows(big), feats[big])


def test_native_stream_file(toy):
    from cmve.linas.bigfile import StreamFile
    d, names, feats, _ = toy
    sf = StreamFile(d, chunk=100)
    got = list(sf)
    assert [n for n, _ in got] == names
    assert np.array_equal(np.asarray([v for _, v in got], np.float32), feats)


def test_native_reader_errors(toy, tmp_path):
    from cmve.linas.bigfile import BigFile
    from cmve._lib import CmveError
    d, names, feats, _ = toy
    bf = BigFile(d)
    with pytest.raises(CmveError, match="out of range"):
        bf.read_rows([len(names)])
    with pytest.raises(CmveError, match="out of range"):
        bf.read_rows([-1])
    bad = tmp_path / "bad"
    bad.mkdir()
    (bad / "shape.txt").write_text("10 96\n")
    (bad / "id.txt").write_text(" ".join(f"x{i}" for i in range(10)))
    np.zeros((5, 96), np.float32).tofile(str(bad / "feature.bin"))  # too short for shape.txt
    with pytest.raises(CmveError, match="shape.txt says"):
        BigFile(str(bad))


@pytest.mark.gpu
def test_gather_to_hbm(toy):
    from cmve.linas.bigfile import BigFile
    d, names, feats, _ = toy
    bf = BigFile(d)
    rows = np.random.default_rng(1).integers(0, len(names), 7777)
    x = bf.to_device(rows, staging_rows=256)  # many double-buffer rounds
    assert np.array_equal(x.cpu().numpy(), feats[rows])


@pytest.mark.gpu
def test_video_batch_loader_matches_reference_collate(toy, golden):
    from cmve.linas.bigfile import BigFile, VideoBatchLoader, read_dict
    d, _, _, _ = toy
    g = golden("bigfile")
    v2f = read_dict(os.path.join(d, "video2frames.txt"))
    vids = sorted(v2f)
    bf = BigFile(d)
    for b, sel in enumerate(BATCHES):
        ld = VideoBatchLoader(bf, v2f, video_ids=[vids[i] for i in sel], batch_size=len(sel))
        (videos, origin, lengths, mask), idxs, ids = ld.batch(0)
        assert list(ids) == list(g[f"batch{b}_ids"])
        assert lengths == list(g[f"batch{b}_lengths"])
        assert np.array_equal(videos.cpu().numpy(), g[f"batch{b}_videos"])
        assert np.array_equal(mask.cpu().numpy(), g[f"batch{b}_mask"])
        np.testing.assert_allclose(origin.cpu().numpy(), g[f"batch{b}_origin"], rtol=0, atol=2e-6)
