"""Deterministic synthetic inputs shared by the golden-vector script, the tests and bench.py.

numpy ``default_rng(seed)`` (PCG64) streams are stable across numpy versions, so a
fixture can store only the seed + shape of its inputs and the expected outputs.
Configs follow SURVEY.md section 8(d).
"""
from __future__ import annotations

import numpy as np


def c1_embeddings(seed=0, n=1000, d=1024, sigma=10.0):
    """C1 'MSR-VTT 1k-A plumbing': V ~ N(0,1)^{n x d}, C = V + sigma * N(0,1) (fp32),
    ids video{i} / video{i}#0.  Returned as the float64 buffers encode_vid/encode_text
    produce (LINAS-engine/evaluation.py:102)."""
    rng = np.random.default_rng(seed)
    v = rng.standard_normal((n, d), dtype=np.float32)
    c = (v + np.float32(sigma) * rng.standard_normal((n, d), dtype=np.float32)).astype(np.float32)
    video_ids = [f"video{i}" for i in range(n)]
    caption_ids = [f"video{i}#0" for i in range(n)]
    return v.astype(np.float64), c.astype(np.float64), video_ids, caption_ids


def multi_caption_embeddings(seed=5, n_v=200, per=20, d=128, sigma=3.0):
    """v2t multi-GT case: `per` captions per video (msrvtt10k has 20), ids video{i}#{k}."""
    rng = np.random.default_rng(seed)
    v = rng.standard_normal((n_v, d), dtype=np.float32)
    c = np.repeat(v, per, axis=0) + np.float32(sigma) * rng.standard_normal((n_v * per, d), dtype=np.float32)
    video_ids = [f"video{i}" for i in range(n_v)]
    caption_ids = [f"video{i}#{k}" for i in range(n_v) for k in range(per)]
    return v.astype(np.float64), c.astype(np.float32).astype(np.float64), video_ids, caption_ids


def gallery_queries(seed=2, n_v=20000, n_q=16, d=1024, sigma=10.0):
    """inference.py case: fp64 gallery (video_data.pt cache), fp32 caption embeddings."""
    rng = np.random.default_rng(seed)
    g = rng.standard_normal((n_v, d), dtype=np.float32)
    pick = rng.choice(n_v, size=n_q, replace=False)
    q = (g[pick] + np.float32(sigma) * rng.standard_normal((n_q, d), dtype=np.float32)).astype(np.float32)
    return g.astype(np.float64), q, pick


def bench_shard(seed, n_v, d=1024, dtype=np.float32):
    rng = np.random.default_rng(seed)
    return rng.standard_normal((n_v, d), dtype=np.float32).astype(dtype)
