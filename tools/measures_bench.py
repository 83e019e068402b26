"""Non-cosine measures row: time K10 (cmve_pairwise) per metric on the GPU
box, against the reference's own CPU call (scipy cdist for the cal_error branches,
evaluation.py:22-33) on a bounded sample of the same workload.  Prints one JSON line.

Roofline: K10 is fp64-VALU bound (no HBM pressure: each 64 x 64 tile reads 2 x 64 x D elements
for 64 x 64 x D element-pairs).  Per element-pair the inner loop issues n_inst fp64 VALU ops
(SQ_L2/L2: sub + fma = 2; L1: sub + add|.| = 2; ORDER: sub + max + fma = 3; JACCARD: min + max +
add + add = 4).  Peak fp64 VALU issue = 78.6 TFLOP/s (spec) / 2 = 3.93e13 ops/s, so the
element-pair ceiling is 3.93e13 / n_inst per second.
Workload: N_c captions x N_v videos x D (default 20000 x 20000 x 1024, an ActivityNet-scale
gallery scored against its captions), synthetic Gaussian (|.| for jaccard)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "cross-modal-video-engine_amd"), ROOT):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cmve import engine, _lib  # noqa: E402

METRICS = {"sq_l2": (_lib.PW_SQ_L2, 2), "l2": (_lib.PW_L2, 2), "l1": (_lib.PW_L1, 2),
           "order": (_lib.PW_ORDER, 3), "jaccard": (_lib.PW_JACCARD, 4)}
PEAK_OPS = 78.6e12 / 2


def main():
    nc = int(os.environ.get("NC", 20000))
    nv = int(os.environ.get("NV", 20000))
    d = int(os.environ.get("D", 1024))
    reps = int(os.environ.get("REPS", 5))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    c = torch.randn((nc, d), device=dev, dtype=torch.float64, generator=g)
    v = torch.randn((nv, d), device=dev, dtype=torch.float64, generator=g)
    res = {}
    for name, (code, n_inst) in METRICS.items():
        a, b = (c.abs(), v.abs()) if name == "jaccard" else (c, v)
        engine.pairwise(a, b, code)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            out = engine.pairwise(a, b, code)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        epairs = nc * nv * d / (ms * 1e-3)
        res[name] = {"ms": ms, "pairs_per_s": nc * nv / (ms * 1e-3), "element_pairs_per_s": epairs,
                     "fp64_ops_per_s": epairs * n_inst, "roofline_frac": epairs * n_inst / PEAK_OPS}
        del out

    # reference CPU path: scipy cdist (fp64) on a bounded caption sample, the whole gallery
    from scipy.spatial import distance
    cs = c[:int(os.environ.get("CPU_NC", 100))].cpu().numpy()
    vs = v.cpu().numpy()
    cpu = {}
    for name, kw in (("l2", dict(metric="euclidean")), ("l1", dict(metric="minkowski", p=1))):
        t0 = time.perf_counter()
        distance.cdist(cs, vs, **kw)
        t = time.perf_counter() - t0
        cpu[name] = {"pairs_per_s": cs.shape[0] * nv / t, "seconds": t}
    print(json.dumps({
        "metric": "caption-video pairs/sec, non-cosine cal_error measures (K10 cmve_pairwise)",
        "config": {"workload": f"{nc} captions x {nv} videos x {d}-d, fp64 inputs, fp64 accumulation",
                   "reps": reps},
        "dtype": "f64",
        "kernels": res,
        "roofline_peak": {"fp64_valu_ops_per_s": PEAK_OPS, "source": "78.6 TFLOP/s fp64 vector (spec) / 2"},
        "cpu_baseline": {"kind": "reference", "call": "scipy.spatial.distance.cdist (evaluation.py:22-33)",
                         "cores": 1, "sample": f"{cs.shape[0]} captions x {nv} videos x {d}", **cpu},
        "speedup_vs_cpu": {k: res[k]["pairs_per_s"] / cpu[k]["pairs_per_s"] for k in cpu}}))


if __name__ == "__main__":
    main()
