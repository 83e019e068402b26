"""inference.py regime (one caption x a 1M-video gallery, exact top-10): per-call wall time and,
under rocprofv3 --kernel-trace --stats, the per-kernel split (GEMV / histogram / collect / finish).
  python tools/gemv_bench.py [--ng N] [--nq 1] [--reps R]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cross-modal-video-engine_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from cmve import engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ng", type=int, default=1048576)
    ap.add_argument("--nq", type=int, default=1)
    ap.add_argument("--d", type=int, default=1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(77)
    gal = torch.randn((a.ng, a.d), generator=gen, device=dev)
    g = engine.RowSet(gal, eps=0.0, with_lo=False, device=dev)
    caps = gal[:a.nq] + 10.0 * torch.randn((a.nq, a.d), generator=gen, device=dev)
    q = engine.RowSet(caps, eps=0.0, with_lo=False, device=dev)
    ws = torch.empty(engine.topk_workspace_floats(q, g, a.k), dtype=torch.float32, device=dev)
    for _ in range(3):
        engine.topk(q, g, a.k, scores_ws=ws, to_host=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        engine.topk(q, g, a.k, scores_ws=ws, to_host=False)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.reps * 1e3
    print(json.dumps({"ng": a.ng, "nq": a.nq, "k": a.k, "ms_per_call_device_resident": ms,
                      "gallery_GBps": a.ng * g.d_pad * 2 / (ms * 1e-3) / 1e9}))


if __name__ == "__main__":
    main()
