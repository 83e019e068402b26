"""Kernel study of the K14 evaluation: s_memrealtime stamps (100 MHz) per block of the three launches
(CMVE_EVAL_DBG=128, a diagnostic mode: timings only).  Prints, per launch, the spread of block starts,
the per-block work time, the last block's tail and the gaps between launches, in microseconds."""
import ctypes
import json
import os
import sys

os.environ["CMVE_EVAL_DBG"] = "128"
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
    buf = np.zeros(3 * 1024 * 4, np.uint64)
    res = []
    for it in range(30):
        buf[:] = 0
        torch.cuda.synchronize()
        sess.enqueue(ct, vt)
        torch.cuda.synchronize()
        _lib.check(f(buf.ctypes.data, buf.nbytes))
        st = buf.reshape(3, 1024, 4).astype(np.int64)
        t_ref = st[0][st[0][:, 0] > 0, 0].min()
        out = {}
        for k, name in enumerate(("prep", "gemm", "fix")):
            s = st[k]
            live = s[:, 0] > 0
            if not live.any():  # the rank GEMM carries no stamps
                continue
            s = s[live]
            rel = (s - t_ref) * 0.01  # us
            d = {"blocks": int(live.sum()), "start_first": float(rel[:, 0].min()), "start_last": float(rel[:, 0].max()),
                 "work_med": float(np.median(rel[:, 1] - rel[:, 0])), "work_max": float((rel[:, 1] - rel[:, 0]).max())}
            ends = rel[:, 3] if k == 1 else rel[:, 1]
            d["work_end_last"] = float(ends.max()) if k != 1 else float(rel[:, 3].max())
            tail = s[s[:, 2] >= s[:, 0].min()]  # this evaluation's last block (older stamps linger)
            if k != 1 and len(tail):
                tr = (tail - t_ref) * 0.01
                d["tail_start"] = float(tr[0, 2])
                d["tail_end"] = float(tr[0, 3])
            if k == 1:
                d["reduce_med"] = float(np.median(rel[:, 2] - rel[:, 1]))
                d["epi_med"] = float(np.median(rel[:, 3] - rel[:, 2]))
            out[name] = d
        res.append(out)
    last = res[-1]
    print(json.dumps(last, indent=1))
    med = {k: {kk: float(np.median([r[k][kk] for r in res])) for kk in res[-1][k]} for k in res[-1]}  # noqa: E501
    print("median over 30 evaluations:", json.dumps(med))


if __name__ == "__main__":
    main()
