"""Calibrate the CPU baseline's oracle port against the imported reference (BASELINE.md section 2:
within +-10 %), in the build container (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tools/calibrate_port.py /root/reference

The timed unit is the bench's cpu_baseline unit: one MSR-VTT-1kA evaluation on the C1 inputs
(tests/golden/synth.py) = cal_error (LINAS-engine/evaluation.py:17-21) + eval_q2m t2v and v2t
(LINAS-engine/util/metrics.py:124-157), run by the reference's own functions and by
oracle/retrieval.py, interleaved, same process, same BLAS threads.  Writes
profiles/r02_cpu_calibration.json."""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT))


def main(ref_root, reps=15):
    sys.path.insert(0, os.path.join(ref_root, "LINAS-engine"))
    import evaluation  # reference
    from util import metrics  # reference
    import synth
    from oracle import retrieval as R
    sys.path.insert(0, ROOT)
    from bench import cpu_info  # noqa: E402  (CPU model / BLAS threads, as the bench reports them)

    v, c, vid, cid = synth.c1_embeddings()
    v2t_gt, t2v_gt = metrics.get_gt(vid, cid)
    t2v_lists = [t2v_gt[i] for i in range(len(cid))]

    def ref_eval():
        e = evaluation.cal_error(v, c, "cosine")
        return metrics.eval_q2m(e, t2v_lists), metrics.eval_q2m(e.T, v2t_gt)

    def port_eval():
        e = R.cal_error(v, c)
        return R.eval_q2m(e, t2v_lists), R.eval_q2m(e.T, v2t_gt)

    assert ref_eval() == port_eval(), "the port's R@K differ from the reference's"
    t_ref, t_port = [], []
    for _ in range(reps):  # interleaved, so drift hits both alike
        t0 = time.perf_counter()
        ref_eval()
        t_ref.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        port_eval()
        t_port.append(time.perf_counter() - t0)
    mr, mp = float(np.median(t_ref)), float(np.median(t_port))
    out = {"unit": "one MSR-VTT-1kA evaluation (1000 x 1000 x 1024: cal_error + eval_q2m t2v + v2t)",
           "reference_ms_median": mr * 1e3, "port_ms_median": mp * 1e3, "port_over_reference": mp / mr,
           "within_10pct": bool(abs(mp / mr - 1.0) <= 0.10), "reps": reps,
           "same_results": True, "host": cpu_info(),
           "note": "build container (the reference is importable only here); bench.py times the port on the "
                   "GPU box's host"}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "r02_cpu_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
