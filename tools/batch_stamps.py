"""Kernel study of a K14 batch (cmve_eval_batch_*): s_memrealtime stamps (100 MHz) of every rank tile of the
batch's evaluations (a diagnostic build: make study NAME=stamps DEFS=-DCMVE_EVAL_DBG=128, loaded with CMVE_LIB=.../libcmve_stamps.so; timings only) plus the first evaluation's prep and
finish blocks.  Prints medians over 20 batch runs: the launch spans, the per-tile phase durations and the
tile duration percentiles, in microseconds from the first prep block's start."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "cross-modal-video-engine_amd"), ROOT, os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import bench
    from cmve import _lib, engine
    K = int(os.environ.get("STAMPS_BATCH", "8"))
    dev = torch.device("cuda", 0)
    sessions, inputs = [], []
    for j in range(K):
        sess, ct, vt, _ = bench.c1_session(dev, seed=j)
        sessions.append(sess)
        inputs.append((ct, vt))
    for s, (c, v) in zip(sessions, inputs):
        s.run(c, v)  # sizes the undecided-pair lists
    rb = engine.RankBatch(sessions, inputs)
    f = _lib.lib.cmve_eval_debug_stamps
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]
    buf = np.zeros(4 * 1024 * 8, np.uint64)
    res = []
    for it in range(23):
        buf[:] = 0
        torch.cuda.synchronize()
        rb.run()
        torch.cuda.synchronize()
        if it < 3:
            continue
        _lib.check(f(buf.ctypes.data, buf.nbytes))
        st = buf.reshape(4, 1024, 8).astype(np.int64)
        t_ref = st[0][st[0][:, 0] > 0, 0].min()
        out = {}
        g = st[3]
        live = g[:, 0] > 0
        rel = (g[live] - t_ref) * 0.01
        dur = rel[:, 3] - rel[:, 0]
        out["gemm"] = {"tiles": int(live.sum()), "start_first": float(rel[:, 0].min()),
                       "start_last": float(rel[:, 0].max()), "end_last": float(rel[:, 3].max()),
                       "tile_p10": float(np.percentile(dur, 10)), "tile_p50": float(np.percentile(dur, 50)),
                       "tile_p90": float(np.percentile(dur, 90))}
        for a, b, nm in ((0, 1, "setup"), (1, 2, "loop"), (2, 4, "publish"), (4, 5, "score"), (5, 6, "emit"),
                         (6, 3, "flush")):
            out["gemm"][nm + "_med"] = float(np.median(rel[:, b] - rel[:, a]))
        # tiles in flight over the launch (sampled every 0.5 us)
        ts = np.arange(rel[:, 0].min(), rel[:, 3].max(), 0.5)
        inflight = ((rel[:, 0][None, :] <= ts[:, None]) & (rel[:, 3][None, :] > ts[:, None])).sum(1)
        out["gemm"]["inflight_med"] = float(np.median(inflight))
        out["gemm"]["inflight_max"] = float(inflight.max())
        for k, name in ((0, "prep"), (1, "finish"), (2, "fix")):
            s = st[k]
            lv = s[:, 0] > 0
            if not lv.any():
                continue
            r2 = (s[lv] - t_ref) * 0.01
            out[name] = {"blocks": int(lv.sum()), "start_first": float(r2[:, 0].min()),
                         "start_last": float(r2[:, 0].max()), "end_last": float(r2[:, 1].max()),
                         "work_med": float(np.median(r2[:, 1] - r2[:, 0]))}
        res.append(out)
    med = {k: {kk: float(np.median([r[k][kk] for r in res])) for kk in res[-1][k]} for k in res[-1]}
    print(f"batch of {K}, median over {len(res)} runs:", json.dumps(med, indent=1))
    rb.close()


if __name__ == "__main__":
    main()
