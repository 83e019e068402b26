"""Developer benchmark of the K14 evaluation (cmve_eval_ranks) on the C1 / MSR-VTT-1kA problem:
per-launch times from the handle's events and the wall time per pipelined evaluation.
    python tools/eval_bench.py [--reps 200] [--dtype f64|f32]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "cross-modal-video-engine_amd"), ROOT, os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--dtype", default="f64")
    a = ap.parse_args()
    import bench
    from cmve import _lib
    dev = torch.device("cuda", 0)
    sess, ct, vt, _ = bench.c1_session(dev)
    if a.dtype == "f32":
        from cmve import engine
        ct, vt = ct.float(), vt.float()
        sess = engine.RankSession(1000, 1000, 1024, row_gts=[[i] for i in range(1000)],
                                  col_gts=[[i] for i in range(1000)], dtype=torch.float32, device=dev)
    t2v, v2t = sess.run(ct, vt)
    for _ in range(10):
        sess.enqueue(ct, vt)
    torch.cuda.synchronize()
    ms = []
    for r in range(a.reps):
        sess.enqueue(ct, vt, timing_slot=r % _lib.EVAL_TIMING_SLOTS)
        if r % _lib.EVAL_TIMING_SLOTS == _lib.EVAL_TIMING_SLOTS - 1:
            ms += [sess.timing(s) for s in range(_lib.EVAL_TIMING_SLOTS)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(a.reps):
        sess.enqueue(ct, vt)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.reps * 1e3
    ms = np.array(ms)
    print(json.dumps({"dtype": a.dtype, "wall_ms_per_eval_no_events": wall,
                      "median_ms": {"prep": float(np.median(ms[:, 0])), "rank_gemm": float(np.median(ms[:, 1])),
                                    "fix_ranks": float(np.median(ms[:, 2]))},
                      "t2v_r1": float(np.mean(t2v <= 1) * 100), "undecided": int(sess.host[8])}))


if __name__ == "__main__":
    main()
