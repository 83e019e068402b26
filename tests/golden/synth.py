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


def multifusion_ranking_case(tsv_rows, n_gallery=2048, d=640, frames=8, seed=3, sigma=7.0):
    """(ix) MultiFusion ranking fixture inputs: the first triplets of the shipped val split
    (idx, ref, target, ...) and a sub-gallery of `n_gallery` integer video names containing every
    ref/target, with synthetic CLIP-like high features [n_gallery, frames, d] and predictions =
    normalize(mean_f(target features) + sigma * noise).  Query 5's target is set to its reference
    (the 'never retrieved' quirk of MultiFusion/src/validate.py:76-83)."""
    rng = np.random.default_rng(seed)
    refs = [int(r[1]) for r in tsv_rows]
    tgts = [int(r[2]) for r in tsv_rows]
    if len(tgts) > 5:
        tgts[5] = refs[5]
    need = sorted(set(refs) | set(tgts))
    pool = np.setdiff1d(np.arange(44493), need)
    extra = rng.choice(pool, size=n_gallery - len(need), replace=False)
    names = np.array(sorted(set(need) | set(extra.tolist())), np.int64)
    feats = rng.standard_normal((n_gallery, frames, d), dtype=np.float32)
    pos = {int(n): i for i, n in enumerate(names)}
    tmean = feats[[pos[t] for t in tgts]].mean(axis=1)
    pred = tmean / np.linalg.norm(tmean, axis=1, keepdims=True) + sigma * rng.standard_normal(tmean.shape).astype(
        np.float32) / np.sqrt(d)
    pred = (pred / np.linalg.norm(pred, axis=1, keepdims=True)).astype(np.float32)
    return names, feats, pred, refs, tgts


COMBINER_SHAPES = [
    ("text_projection_layer.weight", (2560, 640)), ("text_projection_layer.bias", (2560,)),
    ("image_projection_layer.weight", (2560, 640)), ("image_projection_layer.bias", (2560,)),
    ("combiner_layer.weight", (5120, 5120)), ("combiner_layer.bias", (5120,)),
    ("output_layer.weight", (640, 5120)), ("output_layer.bias", (640,)),
    ("dynamic_scalar.0.weight", (5120, 5120)), ("dynamic_scalar.0.bias", (5120,)),
    ("dynamic_scalar.3.weight", (1, 5120)), ("dynamic_scalar.3.bias", (1,)),
    ("m_remained.weight", (640, 640, 1, 1)), ("m_remained.bias", (640,)),
    ("m_residual.weight", (640, 640)), ("m_residual.bias", (640,)),
    ("self_attn_1.attn.in_proj_weight", (1920, 640)), ("self_attn_1.attn.in_proj_bias", (1920,)),
    ("self_attn_1.attn.out_proj.weight", (640, 640)), ("self_attn_1.attn.out_proj.bias", (640,)),
    ("self_attn_1.ln_1.weight", (640,)), ("self_attn_1.ln_1.bias", (640,)),
    ("self_attn_1.mlp.c_fc.weight", (2560, 640)), ("self_attn_1.mlp.c_fc.bias", (2560,)),
    ("self_attn_1.mlp.c_proj.weight", (640, 2560)), ("self_attn_1.mlp.c_proj.bias", (640,)),
    ("self_attn_1.ln_2.weight", (640,)), ("self_attn_1.ln_2.bias", (640,)),
]


def combiner_shapes(d, proj, hidden):
    """COMBINER_SHAPES for Combiner(d, proj, hidden) (the same state-dict order)."""
    sub = {640: d, 2560: proj, 5120: hidden, 1920: 3 * d}
    out = []
    for name, shape in COMBINER_SHAPES:
        if name.startswith("self_attn_1.mlp"):  # the block's MLP is 4 * d wide, not proj
            shape = tuple(4 * d if x == 2560 else d for x in shape)
        else:
            shape = tuple(sub.get(x, x) for x in shape)
        out.append((name, shape))
    return out


def combiner_state(seed=11, dims=(640, 2560, 5120)):
    """Deterministic Combiner(640, 2560, 5120) weights (64.7M params) in state-dict order:
    weights ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (torch's default Linear init range), biases
    ~ 0.05 N(0,1), LayerNorm gain 1 + 0.1 N(0,1).  Both the golden script (loading them into the
    reference module) and the GPU test regenerate them, so no checkpoint is stored.  ``dims`` =
    (clip_feature_dim, projection_dim, hidden_dim) for a smaller Combiner."""
    rng = np.random.default_rng(seed)
    sd = {}
    shapes = COMBINER_SHAPES if tuple(dims) == (640, 2560, 5120) else combiner_shapes(*dims)
    for name, shape in shapes:
        if name.endswith("ln_1.weight") or name.endswith("ln_2.weight"):
            v = 1.0 + 0.1 * rng.standard_normal(shape, dtype=np.float32)
        elif name.endswith("bias"):
            v = 0.05 * rng.standard_normal(shape, dtype=np.float32)
        else:
            fan_in = int(np.prod(shape[1:]))
            bound = 1.0 / np.sqrt(fan_in)
            v = rng.uniform(-bound, bound, size=shape).astype(np.float32)
        sd[name] = v.astype(np.float32)
    return sd


def combiner_inputs(b, seed, frames=8, tokens=16, d=640):
    """ref high [b, f, d], ref middle [b, f, l, d], text [b, d], target high [b, f, d] (fp32)."""
    rng = np.random.default_rng(seed)
    high = rng.standard_normal((b, frames, d), dtype=np.float32)
    mid = rng.standard_normal((b, frames, tokens, d), dtype=np.float32)
    text = rng.standard_normal((b, d), dtype=np.float32)
    tgt = rng.standard_normal((b, frames, d), dtype=np.float32)
    return high, mid, text, tgt


def bigfile_toy(datadir, seed=21, n_videos=40, dim=96):
    """A BigFile directory (shape.txt, id.txt, feature.bin, video2frames.txt) in the layout
    LINAS writes (basic/bigfile.py:6-18, util/get_frameInfo.py:36-52): frame ids
    '<video>_<frame no>' stored in SHUFFLED file order, 1..80 frames per video (some over
    VIDEO_MAX_LEN=64), a few rows belonging to no video.  Returns (names, feats, video2frames)."""
    import os
    rng = np.random.default_rng(seed)
    os.makedirs(datadir, exist_ok=True)
    counts = rng.integers(1, 81, size=n_videos)
    counts[0], counts[1] = 1, 80
    frames = [f"vid{v:03d}_{k}" for v in range(n_videos) for k in range(1, int(counts[v]) + 1)]
    frames += [f"orphan_{k}" for k in range(5)]
    names = [frames[i] for i in rng.permutation(len(frames))]
    feats = rng.standard_normal((len(names), dim), dtype=np.float32)
    with open(os.path.join(datadir, "shape.txt"), "w") as f:
        f.write("%d %d\n" % (len(names), dim))
    with open(os.path.join(datadir, "id.txt"), "w") as f:
        f.write(" ".join(names))
    feats.tofile(os.path.join(datadir, "feature.bin"))
    video2frames = {f"vid{v:03d}": [f"vid{v:03d}_{k}" for k in range(1, int(counts[v]) + 1)]
                    for v in range(n_videos)}
    with open(os.path.join(datadir, "video2frames.txt"), "w") as f:
        f.write(str(video2frames))
    return names, feats, video2frames


BIGFILE_REQUESTS = [
    ["vid003_2", "vid000_1", "nope", "vid003_2", "orphan_4"],   # duplicate + unknown name
    ["vid001_%d" % k for k in range(80, 0, -3)],              # reverse order
]


def multifusion_query(seed=31, frames=8, channels=1280, n_gallery=200, d=640):
    """One composed query of MultiFusion/src/inference.py:124-136: reference high features [f, d],
    middle tokens [f, 18*18, channels], the CLIP text feature [1, d], the target videos' high
    features [n_gallery, f, d] and their paths (fp32)."""
    rng = np.random.default_rng(seed)
    high = rng.standard_normal((frames, d), dtype=np.float32)
    mid = rng.standard_normal((frames, 18 * 18, channels), dtype=np.float32)
    text = rng.standard_normal((1, d), dtype=np.float32)
    gallery = rng.standard_normal((n_gallery, frames, d), dtype=np.float32)
    names = [f"../dataset/videos/V{i:04d}.mp4" for i in range(n_gallery)]
    return high, mid, text, gallery, names
