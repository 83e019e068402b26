#!/bin/bash
# C4 at its configured size under one FETCH_SIZE pass: the fix-up / rank GEMM / attention kernels' fetched bytes
# (2 x FETCH_SIZE: the gfx950 half-count) and durations, last launches of each
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
mkdir -p "$R/gpurun_out/fxp" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/fxp/fetch" -o run -- python3 "$R/tools/fusion_bench.py" --loop-q 0 --sample 16 > "$R/gpurun_out/fxp/fetch.log" 2>&1 || { tail -5 "$R/gpurun_out/fxp/fetch.log"; exit 1; }
python3 - "$R/gpurun_out/fxp" <<'PY'
import collections, csv, glob, sys
f = glob.glob(sys.argv[1] + "/fetch/**/*counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if r["Counter_Name"] == "FETCH_SIZE":
        d[r["Kernel_Name"][:50]].append((float(r["Counter_Value"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
for k, v in d.items():
    if "fixup" in k or "sim_kernel<2" in k or "mha" in k:
        for x in v[-3:]:
            print(k, "fetched GB %.2f" % (2 * x[0] * 1024 / 1e9), "ms %.3f" % x[1])
PY
