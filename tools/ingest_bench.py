"""C5 gallery ingest on one MI355X (MCT/mmaction/models/recognizers/recognizer2d.py:76-83
-> LINAS Latent_mapping-style projection -> l2norm -> packed gallery): TSN segment features
[N, 25, 2048] fp32 resident in HBM -> segment mean (K2) -> Linear 2048 -> 1024 (K3, split-bf16)
-> L2 + pack into the fp16 / bf16 planes the rank and top-k kernels read (K1).  Per-stage device
times (HIP events) and the HBM roofline of the pool (the dominant byte stream).  Random-init
weights, synthetic features.  Prints one JSON line.   python tools/ingest_bench.py [--n N]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cross-modal-video-engine_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from cmve import engine  # noqa: E402
from cmve.linas.model import temporal_pool, linear_fused, _PackedWeight  # noqa: E402

PEAK_HBM_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=131072, help="videos (one 8-GPU shard of the 1M gallery)")
    ap.add_argument("--segs", type=int, default=25)
    ap.add_argument("--feat", type=int, default=2048)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--chunk", type=int, default=32768)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(4)
    feats = torch.randn((a.n, a.segs, a.feat), generator=gen, device=dev)
    torch.manual_seed(0)
    fc = torch.nn.Linear(a.feat, a.dim).to(dev)
    pw = _PackedWeight()
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

    def run():
        t = {"pool": 0.0, "project": 0.0, "pack": 0.0}
        sets = []
        for c0 in range(0, a.n, a.chunk):
            e = [ev() for _ in range(4)]
            e[0].record()
            pooled = temporal_pool(feats[c0:c0 + a.chunk], "mean")
            e[1].record()
            emb = linear_fused(pooled, fc.weight, fc.bias, packed=pw)
            e[2].record()
            sets.append(engine.RowSet(emb, eps=0.0, with_lo=False, device=dev))
            e[3].record()
            torch.cuda.synchronize()
            t["pool"] += e[0].elapsed_time(e[1])
            t["project"] += e[1].elapsed_time(e[2])
            t["pack"] += e[2].elapsed_time(e[3])
        return t, sets

    run()
    times = [run()[0] for _ in range(a.reps)]
    med = {k: float(np.median([t[k] for t in times])) for k in times[0]}
    total = sum(med.values())
    pool_bytes = a.n * a.segs * a.feat * 4 + a.n * a.feat * 4
    flops = 2.0 * a.n * a.feat * a.dim
    out = {"videos": a.n, "segments": a.segs, "feat": a.feat, "dim": a.dim, "ms": med, "total_ms": total,
           "videos_per_s": a.n / (total * 1e-3),
           "pool_roofline": {"bound": "hbm", "achieved_GBps": pool_bytes / (med["pool"] * 1e-3) / 1e9,
                             "peak_GBps": PEAK_HBM_GBS,
                             "frac": pool_bytes / (med["pool"] * 1e-3) / 1e9 / PEAK_HBM_GBS},
           "project_tflops_algorithmic": flops / (med["project"] * 1e-3) / 1e12,
           "note": "projection in split-bf16 (3 MFMAs per product); pack = fp64 norm + fp16 / bf16 planes + bounds"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
