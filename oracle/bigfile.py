"""TEST INFRASTRUCTURE ONLY (checker, never shipped): CPU restatement of LINAS's BigFile reader.

read(): LINAS-engine/basic/bigfile.py:23-56 -- requested ids de-duplicated, unknown names dropped,
sorted by row, rows read with seek + fromfile, returned as (names, list-of-lists).
read_dict(): basic/util.py:77-82 (the reference evals the dict literal; literal_eval is equivalent
on the files util/get_frameInfo.py:36-52 writes).
collate(): tag_data_provider.py:91-109 over VisDataSet4DualEncoding items (:330-337).
Pinned by tests/golden/bigfile.npz (produced by running the reference modules,
tests/golden/make_golden_bigfile.py)."""
from __future__ import annotations

import ast
import os

import numpy as np

VIDEO_MAX_LEN = 64


class BigFileOracle:
    def __init__(self, datadir):
        with open(os.path.join(datadir, "shape.txt")) as f:
            self.n, self.d = map(int, f.readline().split())
        with open(os.path.join(datadir, "id.txt"), "rb") as f:
            self.names = [str(x, encoding="ISO-8859-1") for x in f.read().strip().split()]
        self.name2index = dict(zip(self.names, range(self.n)))
        self.path = os.path.join(datadir, "feature.bin")

    def read(self, requested, isname=True):
        requested = set(requested)
        if isname:
            pairs = [(self.name2index[x], x) for x in requested if x in self.name2index]
        else:
            pairs = [(x, self.names[x]) for x in requested]
        if not pairs:
            return [], []
        pairs.sort(key=lambda v: v[0])
        vecs = []
        with open(self.path, "rb") as f:
            for r, _ in pairs:
                f.seek(r * 4 * self.d)
                vecs.append(np.fromfile(f, dtype=np.float32, count=self.d).tolist())
        return [p[1] for p in pairs], vecs

    def read_one(self, name):  # bigfile.py:58-60
        return self.read([name])[1][0]


def read_dict(path):
    with open(path) as f:
        return ast.literal_eval(f.read())


def collate(frames_list):
    """collate_frame over [frames[T_i, F]] -> (videos, origin, lengths, mask) as numpy."""
    lengths = [min(VIDEO_MAX_LEN, len(f)) for f in frames_list]
    F = len(frames_list[0][0])
    B, t_max = len(frames_list), max(lengths)
    videos = np.zeros((B, t_max, F), np.float32)
    origin = np.zeros((B, F), np.float32)
    mask = np.zeros((B, t_max), np.float32)
    for i, fr in enumerate(frames_list):
        fr = np.asarray(fr, np.float32)
        videos[i, :lengths[i]] = fr[:lengths[i]]
        origin[i] = fr.mean(0)
        mask[i, :lengths[i]] = 1.0
    return videos, origin, lengths, mask
