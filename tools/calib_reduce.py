"""Reduce the calibration passes of tools/calib.sh: per launch of tools/calib.py's schedule, the counter value
(rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB) over the known byte count.
    python tools/calib_reduce.py <outdir>   -> <outdir>/calib.json"""
import csv
import glob
import json
import os
import sys


def counters(path, name):
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r.get("Counter_Name") == name]
    per = {}
    for r in rows:
        k = r["Kernel_Name"]
        if not any(n in k for n in ("read16_kernel", "read_prep_kernel", "write8_kernel", "write16_kernel")):
            continue
        did = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
        per.setdefault(did, [k, 0.0])[1] += float(r["Counter_Value"])
    return [per[d] for d in sorted(per)]


def main(out):
    sched = json.load(open(os.path.join(out, "schedule.json")))
    res = {}
    for cname, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        got = counters(os.path.join(out, sub), cname)
        lines = []
        for i, (s, g) in enumerate(zip(sched, got)):
            lines.append({"launch": i, "kernel": s["kernel"], "bytes": s["bytes"], "counter_kib": g[1],
                          "counter_bytes_over_bytes": g[1] * 1024 / s["bytes"], "trace_kernel": g[0][:60]})
        res[cname] = lines
    json.dump(res, open(os.path.join(out, "calib.json"), "w"), indent=1)
    for k, v in res.items():
        for l in v:
            print(k, l["launch"], l["kernel"], l["bytes"], round(l["counter_bytes_over_bytes"], 4))


if __name__ == "__main__":
    main(sys.argv[1])
