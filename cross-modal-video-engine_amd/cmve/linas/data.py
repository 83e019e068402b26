"""Mirror of ``collate_frame`` (LINAS-engine/util/tag_data_provider.py:91-109) on libcmve.so.

Same input (list of ``(frames[T_i, F], idx, video_id)``) and output
``((videos[B, T_max, F], videos_origin[B, F], lengths, videos_mask[B, T_max]), idxs, video_ids)``;
the pad/truncate to VIDEO_MAX_LEN=64 and the mean over ALL frames run in one HBM-bound
kernel (K2) and the tensors are returned on the GPU (embed_vis moves them there anyway,
LINAS-engine/model.py:711-722).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import engine
from .._lib import lib, check

VIDEO_MAX_LEN = 64  # tag_data_provider.py:11


def collate_frame(data, device=None):
    videos, idxs, video_ids = zip(*data)
    device = device or engine.default_device()
    lengths = [min(VIDEO_MAX_LEN, len(f)) for f in videos]
    F = len(videos[0][0])
    B = len(videos)
    t_max = max(lengths)
    T = np.fromiter((len(f) for f in videos), np.int64, count=B)
    off = np.zeros(B + 1, np.int64)
    np.cumsum(T, out=off[1:])
    frames = torch.cat([torch.as_tensor(f, dtype=torch.float32) for f in videos], 0).to(device).contiguous()
    offt = torch.from_numpy(off).to(device)
    vids = torch.empty((B, t_max, F), dtype=torch.float32, device=device)
    origin = torch.empty((B, F), dtype=torch.float32, device=device)
    mask = torch.empty((B, t_max), dtype=torch.float32, device=device)
    check(lib.cmve_collate_frames(engine.handle(device), engine._ptr(frames), frames.stride(0), engine._ptr(offt),
                                  B, F, VIDEO_MAX_LEN, t_max, engine._ptr(vids), engine._ptr(origin),
                                  engine._ptr(mask)), "cmve_collate_frames")
    return (vids, origin, lengths, mask), idxs, video_ids
