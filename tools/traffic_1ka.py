"""Reduce the rocprofv3 passes of tools/profile_1ka.sh to per-launch figures of the four K14
evaluation launches (pack + GT scores, rank GEMM, fix-up, ranks + R@K) of the 1k-A headline.

HBM bytes per dispatch = 2 * FETCH_SIZE(KiB) * 1024 + WRITE_SIZE(KiB) * 1024 (gfx950 FETCH_SIZE
half-count on wide reads, MI355X_MICROARCH.md).  Writes profiles/<tag>_1ka_traffic.json (read by
bench.py) and copies the kernel-stats summary to profiles/<tag>_1ka_kernel_stats.csv.
    python tools/traffic_1ka.py <outdir> <tag>"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


ROLES = ("pack_gt_scores", "rank_gemm", "fixup", "ranks_recall")


def role(name):
    """The evaluation launch a kernel name is; the batch kernels (cmve_eval_batch_*: the headline's timed loop)
    and the single-evaluation kernels (cmve_eval_ranks: the bench's latency measurements) are kept apart, so a
    profile holding both never averages one into the other."""
    # sim_kernel<MODE, EPI, WM, WN, TM, PHASED, BATCH, KG> (round 6 added KG; earlier traces end at BATCH)
    batch = "_batch_kernel" in name or ("sim_kernel<2, 1" in name and (", true>" in name or ", true, 1>" in name))
    if "eval_prep_kernel" in name or "eval_prep_pair_kernel" in name or "eval_prep_pair_batch_kernel" in name \
            or "eval_prep_fin_batch_kernel" in name \
            or "eval_prep_batch_kernel" in name or "eval_prep_pair_f16_kernel" in name \
            or "eval_prep_pair_f16_batch_kernel" in name:
        r = "pack_gt_scores"
    elif "eval_fix_kernel" in name or "eval_fix_batch_kernel" in name:
        r = "fixup"
    elif "eval_finish_kernel" in name or "eval_finish_batch_kernel" in name:
        r = "ranks_recall"
    elif "sim_kernel<2, 1" in name:
        r = "rank_gemm"
    else:
        return None
    return r if batch else r + "_single"


def main(outdir, tag):
    prof = os.path.join(outdir, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(outdir, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_1ka_kernel_stats.csv"))
    per = defaultdict(lambda: defaultdict(list))
    for counter, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        for r in rows(os.path.join(outdir, sub, "**", "*counter_collection.csv")):
            k = role(r.get("Kernel_Name", ""))
            if k and r.get("Counter_Name") == counter:
                per[k][counter].append(float(r["Counter_Value"]))
    # the counter passes are kernel traces of the same command too: their per-launch durations beside the trace's
    pdur = defaultdict(list)
    for r in rows(os.path.join(outdir, "fetch", "**", "*counter_collection.csv")):
        k = role(r.get("Kernel_Name", ""))
        if k and r.get("Counter_Name") == "FETCH_SIZE":
            pdur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    sq = defaultdict(lambda: defaultdict(list))
    for r in rows(os.path.join(outdir, "sq", "**", "*counter_collection.csv")):
        k = role(r.get("Kernel_Name", ""))
        if k:
            sq[k][r.get("Counter_Name")].append(float(r["Counter_Value"]))
    dur, evals = defaultdict(list), defaultdict(list)
    for r in rows(os.path.join(outdir, "trace", "**", "*kernel_trace.csv")):
        k = role(r.get("Kernel_Name", ""))
        if k:
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
            evals[k].append(int(r.get("Grid_Size_Y") or 1))  # batches: grid y = the evaluations
    kernels = {}
    batch_mode = any(len(dur[k]) for k in ROLES)
    roles = ROLES if batch_mode else tuple(k + "_single" for k in ROLES)
    for k in ROLES + tuple(k + "_single" for k in ROLES):
        f, w = per[k]["FETCH_SIZE"], per[k]["WRITE_SIZE"]
        e = {"launches_traced": len(dur[k]),
             "evaluations_per_launch": (max(set(evals[k]), key=evals[k].count)) if evals[k] else None,
             "trace_avg_ms": (sum(dur[k]) / len(dur[k])) if dur[k] else None,
             "trace_total_ms": sum(dur[k]),
             "fetch_kib_per_launch": (sum(f) / len(f)) if f else None,
             "write_kib_per_launch": (sum(w) / len(w)) if w else None}
        if dur[k]:
            e["trace_median_ms"] = sorted(dur[k])[len(dur[k]) // 2]
        if pdur[k]:
            e["fetch_pass_avg_ms"] = sum(pdur[k]) / len(pdur[k])
        if f and w:
            e["hbm_bytes_per_launch"] = 2 * e["fetch_kib_per_launch"] * 1024 + e["write_kib_per_launch"] * 1024
        if sq[k]:
            med = {c: sorted(v)[len(v) // 2] for c, v in sq[k].items()}
            e["sq_per_launch_median"] = med
            if med.get("SQ_WAVES"):
                e["valu_insts_per_wave"] = med.get("SQ_INSTS_VALU", 0) / med["SQ_WAVES"]
        kernels[k] = e
    dominant = max(roles, key=lambda k: kernels[k]["trace_total_ms"])
    out = {"tag": tag, "workload": "MSR-VTT-1kA exact evaluation, 1000 x 1000 x 1024, float64 inputs",
           "kernels": kernels, "dominant": dominant,
           "hbm_bytes_per_launch": kernels[dominant].get("hbm_bytes_per_launch"),
           "correction": "2 x FETCH_SIZE (gfx950 half-count on wide reads) + WRITE_SIZE, KiB -> bytes"}
    json.dump(out, open(os.path.join(prof, f"{tag}_1ka_traffic.json"), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
