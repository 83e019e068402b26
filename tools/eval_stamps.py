"""Kernel study of the K14 evaluation: s_memrealtime stamps (100 MHz) per block of the prep, fix-up and
finish launches (a diagnostic build: make study NAME=stamps DEFS=-DCMVE_EVAL_DBG=128, loaded with CMVE_LIB; timings only; the rank GEMM carries none).
Prints, per launch, the first / last block start and the first / last block end, in microseconds from
the first prep block's start, median over 30 evaluations."""
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
    from cmve import _lib
    dev = torch.device("cuda", 0)
    sess, ct, vt, _ = bench.c1_session(dev)
    f = _lib.lib.cmve_eval_debug_stamps
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]
    buf = np.zeros(4 * 1024 * 8, np.uint64)
    res = []
    warm = int(os.environ.get("STAMPS_WARM", "0"))  # evaluations enqueued just before the stamped one (GPU busy)
    for it in range(30):
        buf[:] = 0
        torch.cuda.synchronize()
        for _ in range(warm):
            sess.enqueue(ct, vt)
        sess.enqueue(ct, vt)
        torch.cuda.synchronize()
        _lib.check(f(buf.ctypes.data, buf.nbytes))
        st = buf.reshape(4, 1024, 8).astype(np.int64)
        t_ref = st[0][st[0][:, 0] > 0, 0].min()
        out = {}
        g = st[3]
        live = g[:, 0] > 0
        if live.any():
            rel = (g[live] - t_ref) * 0.01
            gm = {"tiles": int(live.sum()), "start_first": float(rel[:, 0].min()), "start_last": float(rel[:, 0].max()),
                  "end_last": float(rel[:, 3].max())}
            for a, b, nm in ((0, 1, "setup"), (1, 2, "loop"), (2, 4, "publish"), (4, 5, "score"), (5, 6, "emit"),
                             (6, 3, "flush")):
                gm[nm + "_med"] = float(np.median(rel[:, b] - rel[:, a]))
            out["gemm"] = gm
        for k, name in ((0, "prep"), (2, "fix"), (1, "finish")):
            s = st[k]
            live = s[:, 0] > 0
            if not live.any():
                continue
            rel = (s[live] - t_ref) * 0.01  # us
            out[name + "_start_pct"] = {f"p{q}": float(np.percentile(rel[:, 0], q)) for q in (10, 50, 90, 99)}
            out[name] = {"blocks": int(live.sum()), "start_first": float(rel[:, 0].min()),
                         "start_last": float(rel[:, 0].max()), "end_first": float(rel[:, 1].min()),
                         "end_last": float(rel[:, 1].max()), "work_med": float(np.median(rel[:, 1] - rel[:, 0]))}
        res.append(out)
    med = {k: {kk: float(np.median([r[k][kk] for r in res])) for kk in res[-1][k]} for k in res[-1]}
    print("median over 30 evaluations:", json.dumps(med, indent=1))


if __name__ == "__main__":
    main()
