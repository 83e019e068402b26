"""Mirror of LINAS's on-disk feature store (``LINAS-engine/basic/bigfile.py``) on libcmve.so.

``BigFile(datadir)`` keeps the reference constructor and ``read`` / ``read_one`` / ``shape``
semantics (names decoded ISO-8859-1, requested ids de-duplicated and returned in file order,
missing names dropped, vectors as Python lists), but ``feature.bin`` is mapped once by
``cmve_bigfile_open`` and rows are gathered natively (``cmve_bigfile_gather``) instead of one
``open`` + ``seek`` + ``array.fromfile`` per call (bigfile.py:23-56).  The array fast paths
``read_rows`` / ``to_device`` skip the list conversion; ``to_device`` streams straight into HBM
through pinned staging (``cmve_bigfile_gather_device``).

``read_dict`` replaces ``basic/util.py:77-82`` (``eval`` of a dict literal) with
``ast.literal_eval``: same result on the literal ``video2frames.txt`` files
(``util/get_frameInfo.py:36-52``), nothing executed.

``VideoBatchLoader`` replaces ``get_vis_data_loader`` + ``VisDataSet4DualEncoding`` +
``collate_frame`` (``util/tag_data_provider.py:91-109,317-342,503-512``): per batch it maps the
videos' frame names to rows, gathers them into HBM and runs the K2 collate there, yielding the
same ``((videos, videos_origin, lengths, videos_mask), idxs, video_ids)`` (tensors on the GPU).
"""
from __future__ import annotations

import ast
import ctypes as C
import os
from typing import Dict, Iterable, List, Sequence

import numpy as np
import torch

from .. import engine
from .._lib import lib, check
from .data import VIDEO_MAX_LEN

_THREADS = int(os.environ.get("CMVE_IO_THREADS", min(16, os.cpu_count() or 1)))


def read_dict(filepath: str) -> dict:
    """basic/util.py:77-82, without executing the file (ast.literal_eval)."""
    with open(filepath, "r") as f:
        return ast.literal_eval(f.read())


class BigFile:
    """basic/bigfile.py:4-62 on a native, mmapped reader."""

    def __init__(self, datadir: str):
        with open(os.path.join(datadir, "shape.txt")) as f:
            self.nr_of_images, self.ndims = map(int, f.readline().split())
        with open(os.path.join(datadir, "id.txt"), "rb") as f:
            self.names = [str(x, encoding="ISO-8859-1") for x in f.read().strip().split()]
        assert len(self.names) == self.nr_of_images
        self.name2index = dict(zip(self.names, range(self.nr_of_images)))
        self.binary_file = os.path.join(datadir, "feature.bin")
        self._h = C.c_void_p()
        check(lib.cmve_bigfile_open(self.binary_file.encode(), self.nr_of_images, self.ndims, C.byref(self._h)),
              "cmve_bigfile_open")
        print("[%s] %dx%d instances loaded from %s" % (self.__class__.__name__, self.nr_of_images, self.ndims,
                                                        datadir))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.cmve_bigfile_close(h)
            self._h = C.c_void_p()

    # ---- array fast paths ----
    def read_rows(self, rows: Sequence[int]) -> np.ndarray:
        """float32 [len(rows), ndims] in the given order (duplicates allowed)."""
        idx = np.ascontiguousarray(np.asarray(rows, dtype=np.int64))
        out = np.empty((idx.size, self.ndims), np.float32)
        if idx.size:
            check(lib.cmve_bigfile_gather(self._h, idx.ctypes.data, idx.size, out.ctypes.data, _THREADS),
                  "cmve_bigfile_gather")
        return out

    def to_device(self, rows: Sequence[int], device=None, staging_rows: int = 4096) -> torch.Tensor:
        """float32 [len(rows), ndims] gathered straight into HBM (pinned double-buffered staging)."""
        device = device or engine.default_device()
        idx = np.ascontiguousarray(np.asarray(rows, dtype=np.int64))
        out = torch.empty((idx.size, self.ndims), dtype=torch.float32, device=device)
        if idx.size:
            staging = torch.empty((max(2, staging_rows), self.ndims), dtype=torch.float32).pin_memory()
            check(lib.cmve_bigfile_gather_device(engine.handle(device), self._h, idx.ctypes.data, idx.size,
                                                 engine._ptr(out), staging.data_ptr(), staging.shape[0], _THREADS),
                  "cmve_bigfile_gather_device")
            torch.cuda.current_stream(device).synchronize()  # staging is freed on return
        return out

    # ---- reference API ----
    def read(self, requested: Iterable, isname: bool = True):
        """bigfile.py:23-56: (names, vectors) for the requested ids, in file order."""
        requested = set(requested)
        if isname:
            index_name_array = [(self.name2index[x], x) for x in requested if x in self.name2index]
        else:
            assert min(requested) >= 0
            assert max(requested) < len(self.names)
            index_name_array = [(x, self.names[x]) for x in requested]
        if len(index_name_array) == 0:
            return [], []
        index_name_array.sort(key=lambda v: v[0])
        vecs = self.read_rows([x[0] for x in index_name_array])
        return [x[1] for x in index_name_array], vecs.tolist()

    def read_one(self, name):
        renamed, vectors = self.read([name])
        return vectors[0]

    def shape(self):
        return [self.nr_of_images, self.ndims]


class StreamFile:
    """bigfile.py:65-103: sequential (id, vector) iteration over the whole file."""

    def __init__(self, datadir: str, chunk: int = 4096):
        self._bf = BigFile(datadir)
        self.nr_of_images, self.ndims = self._bf.nr_of_images, self._bf.ndims
        self.names = self._bf.names
        self.chunk = chunk
        self.current = 0
        self._buf, self._buf0 = None, 0

    def open(self):
        self.current = 0
        self._buf = None

    def close(self):
        self._buf = None

    def __iter__(self):
        return self

    def __next__(self):
        if self.current >= self.nr_of_images:
            self.close()
            raise StopIteration
        if self._buf is None or self.current >= self._buf0 + self._buf.shape[0]:
            self._buf0 = self.current
            self._buf = self._bf.read_rows(range(self.current, min(self.nr_of_images, self.current + self.chunk)))
        v = self._buf[self.current - self._buf0]
        _id = self.names[self.current]
        self.current += 1
        return _id, v.tolist()

    next = __next__


class VideoBatchLoader:
    """get_vis_data_loader + collate_frame (tag_data_provider.py:91-109,317-342,503-512) on the GPU."""

    def __init__(self, vis_feat: BigFile, video2frames: Dict[str, List[str]], video_ids=None,
                 batch_size: int = 100, device=None):
        self.feat = vis_feat
        self.video2frames = video2frames
        self.video_ids = list(video_ids) if video_ids is not None else list(video2frames.keys())
        self.batch_size = batch_size
        self.device = device or engine.default_device()

    def __len__(self):
        return (len(self.video_ids) + self.batch_size - 1) // self.batch_size

    @property
    def dataset(self):
        """The videos in loader order (``len(loader.dataset)`` as evaluation.encode_vid reads it)."""
        return self.video_ids

    def batch(self, b: int):
        vids = self.video_ids[b * self.batch_size:(b + 1) * self.batch_size]
        idxs = tuple(range(b * self.batch_size, b * self.batch_size + len(vids)))
        frames = [self.video2frames[v] for v in vids]
        n2i = self.feat.name2index
        rows = np.fromiter((n2i[f] for fl in frames for f in fl), np.int64, count=sum(len(fl) for fl in frames))
        T = np.fromiter((len(fl) for fl in frames), np.int64, count=len(frames))
        off = np.zeros(len(frames) + 1, np.int64)
        np.cumsum(T, out=off[1:])
        dev = self.device
        x = self.feat.to_device(rows, dev)
        B, F = len(vids), self.feat.ndims
        lengths = [min(VIDEO_MAX_LEN, int(t)) for t in T]
        t_max = max(lengths)
        offt = torch.from_numpy(off).to(dev)
        videos = torch.empty((B, t_max, F), dtype=torch.float32, device=dev)
        origin = torch.empty((B, F), dtype=torch.float32, device=dev)
        mask = torch.empty((B, t_max), dtype=torch.float32, device=dev)
        check(lib.cmve_collate_frames(engine.handle(dev), engine._ptr(x), x.stride(0), engine._ptr(offt), B, F,
                                      VIDEO_MAX_LEN, t_max, engine._ptr(videos), engine._ptr(origin),
                                      engine._ptr(mask)), "cmve_collate_frames")
        return (videos, origin, lengths, mask), idxs, tuple(vids)

    def __iter__(self):
        for b in range(len(self)):
            yield self.batch(b)


def load_video_cache(path: str):
    """inference.py:57-60 ``video_data.pt`` cache {'video_embs', 'video_ids'} (the float64 ndarray
    encode_vid returns and the id list), loaded with ``weights_only=True`` and numpy's array
    reconstruction admitted (no code executed); a cache the safe loader refuses raises."""
    from .checkpoint import _safe_globals
    with torch.serialization.safe_globals(_safe_globals()):
        d = torch.load(path, weights_only=True, map_location="cpu")
    return d["video_embs"], list(d["video_ids"])


def save_video_cache(path: str, video_embs, video_ids):
    """inference.py:67: torch.save({'video_embs', 'video_ids'}) as the reference writes it."""
    torch.save({"video_embs": video_embs, "video_ids": list(video_ids)}, path)
