"""Golden vectors for the on-disk feature-store row, produced by running the
REFERENCE's own modules on the deterministic toy BigFile of synth.bigfile_toy:

  LINAS-engine/basic/bigfile.py:23-60            BigFile.read (by name, by index) / read_one
  LINAS-engine/basic/util.py:77-82               read_dict (video2frames.txt)
  LINAS-engine/util/tag_data_provider.py:317-342 VisDataSet4DualEncoding.__getitem__
  LINAS-engine/util/tag_data_provider.py:91-109  collate_frame

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_bigfile.py /root/reference
Writes tests/golden/bigfile.npz (the toy store itself is regenerated from its seed by the tests).
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import synth  # noqa: E402

BATCHES = [list(range(0, 16)), [1, 0, 7, 39, 12]]  # video indices into sorted video ids


def main(ref_root):
    sys.path.insert(0, os.path.join(ref_root, "LINAS-engine"))
    from basic.bigfile import BigFile  # noqa
    from basic.util import read_dict  # noqa
    from util import tag_data_provider as TDP  # noqa
    out = {}
    with tempfile.TemporaryDirectory() as d:
        synth.bigfile_toy(d)
        bf = BigFile(d)
        for q, req in enumerate(synth.BIGFILE_REQUESTS):
            names, vecs = bf.read(req)
            out[f"read{q}_names"] = np.array(names)
            out[f"read{q}_vecs"] = np.asarray(vecs, np.float32)
        names, vecs = bf.read([5, 2, 2, 0, 17], isname=False)
        out["readidx_names"] = np.array(names)
        out["readidx_vecs"] = np.asarray(vecs, np.float32)
        out["read_one"] = np.asarray(bf.read_one("vid002_1"), np.float32)
        v2f = read_dict(os.path.join(d, "video2frames.txt"))
        vids = sorted(v2f.keys())
        out["video_ids"] = np.array(vids)
        ds = TDP.VisDataSet4DualEncoding(bf, v2f, video_ids=vids)
        for b, sel in enumerate(BATCHES):
            (videos, origin, lengths, mask), idxs, video_ids = TDP.collate_frame([ds[i] for i in sel])
            out[f"batch{b}_videos"] = videos.numpy()
            out[f"batch{b}_origin"] = origin.numpy()
            out[f"batch{b}_lengths"] = np.asarray(lengths, np.int64)
            out[f"batch{b}_mask"] = mask.numpy()
            out[f"batch{b}_ids"] = np.array(video_ids)
    np.savez_compressed(os.path.join(HERE, "bigfile.npz"), **out)
    print("wrote", os.path.join(HERE, "bigfile.npz"), {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
