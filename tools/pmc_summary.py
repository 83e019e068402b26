"""Summarise a tools/pmc.sh output directory: per sim_kernel dispatch, duration and counters."""
import collections
import csv
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "sim_kernel"
rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
tr = {r["Dispatch_Id"]: r for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv"))}
agg = collections.OrderedDict()
for r in rows:
    if pat not in r["Kernel_Name"]:
        continue
    agg.setdefault(r["Dispatch_Id"], collections.defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
for disp, c in agg.items():
    t = tr.get(disp)
    dur = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) * 1e-9 if t else float("nan")
    print(disp, f"{dur * 1e3:.3f} ms", " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))
