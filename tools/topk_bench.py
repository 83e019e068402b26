"""Large-batch exact top-k (C5 regime): cmve_topk_batch (K13, no score matrix) vs the dense
cmve_topk path, 16,384 captions x a 131,072-video shard x 1024-d, k = 10.  Prints one JSON line.
Run on the GPU box: python tools/topk_bench.py [--nq N] [--ng N] [--reps R]"""
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
    p = argparse.ArgumentParser()
    p.add_argument("--nq", type=int, default=16384)
    p.add_argument("--ng", type=int, default=131072)
    p.add_argument("--d", type=int, default=1024)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--no-dense", action="store_true")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(5)
    gal = torch.randn((a.ng, a.d), generator=gen, device=dev)
    pick = torch.randint(0, a.ng, (a.nq,), generator=gen, device=dev)
    qs = gal[pick] + 10.0 * torch.randn((a.nq, a.d), generator=gen, device=dev)
    g = engine.RowSet(gal, eps=0.0, with_lo=True, device=dev)
    q = engine.RowSet(qs, eps=0.0, with_lo=True, device=dev)
    ok, ns, nf = engine.topk_batch_plan(q, g, a.k)
    out = {"nq": a.nq, "ng": a.ng, "d": a.d, "k": a.k, "sample_rows": ns, "batch_ws_GB": nf * 4 / 1e9}
    ws = torch.empty(nf, dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream()

    def timed(fn):
        ts = []
        for r in range(a.reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            res = fn()
            e1.record(s)
            torch.cuda.synchronize()
            if r >= 2:
                ts.append(e0.elapsed_time(e1))
        return float(np.median(ts)), res

    ms_b, (ib, sb, ub) = timed(lambda: engine.topk_batch(q, g, a.k, ws=ws))
    out["batch"] = {"ms": ms_b, "pairs_per_s": a.nq * a.ng / (ms_b * 1e-3), "unresolved": int(ub.item())}
    if not a.no_dense:
        del ws
        torch.cuda.empty_cache()
        need = engine.topk_workspace_floats(q, g, a.k)
        wsd = torch.empty(need, dtype=torch.float32, device=dev)
        ms_d, (id_, sd) = timed(lambda: engine.topk(q, g, a.k, scores_ws=wsd, to_host=False, batch=False))
        out["dense"] = {"ms": ms_d, "pairs_per_s": a.nq * a.ng / (ms_d * 1e-3), "ws_GB": need * 4 / 1e9}
        out["identical"] = bool(torch.equal(ib, id_) and torch.equal(sb, sd))
        out["speedup"] = ms_d / ms_b
    print(json.dumps(out))


if __name__ == "__main__":
    main()
