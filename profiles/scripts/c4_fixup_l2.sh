#!/bin/bash
# C4 fix-up: L2 hit / miss counters, plain vs tiled walk
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/c4_fixup_l2 || exit 1
O=$R/gpurun_out/c4_fixup_l2
cd /tmp && export TMPDIR=/tmp
for g in -1 0 1; do
  CMVE_CIRR_FIX_GROUP=$g timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-trace --output-format csv -d /tmp/l2$g -o run -- python3 "$R/tools/fusion_bench.py" --loop-q 0 --sample 16 > "$O/l2$g.log" 2>&1 || { tail -5 "$O/l2$g.log"; exit 1; }
  python3 - /tmp/l2$g $g <<'PY'
import collections, csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:40]
    if "fixup" in k:
        d[(k, r["Dispatch_Id"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (k, di), v in list(d.items())[-2:]:
    h, m, q = sum(v["TCC_HIT_sum"]), sum(v["TCC_MISS_sum"]), sum(v["TCC_REQ_sum"])
    print("group", sys.argv[2], k, di, "req %.3g hit %.3g miss %.3g hit rate %.3f" % (q, h, m, h / max(1, h + m)))
PY
done
