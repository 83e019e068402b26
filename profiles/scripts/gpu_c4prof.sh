#!/bin/bash
# C4 at its configured size (30,364 queries x 44,493 videos): fusion_bench without the per-batch loop, plain and
# under a rocprofv3 kernel trace -> gpurun_out/<TAG>/{fb.json, trace/}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
TAG=${1:-c4}
cd "$R" && mkdir -p gpurun_out/$TAG || exit 1
O=$R/gpurun_out/$TAG
timeout -k 10 300 python3 tools/fusion_bench.py --loop-q 0 ${FB_ARGS:-} > $O/fb.json 2> $O/fb.err || { tail -20 $O/fb.err; exit 1; }
cat $O/fb.json
[ -n "$NOPROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 "$R/tools/fusion_bench.py" --loop-q 0 ${FB_ARGS:-} > "$O/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$O/trace.log"; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/trace/**/run_kernel_stats.csv", recursive=True)[0]
for x in list(csv.DictReader(open(f)))[:16]:
    print(x["Name"][:100], x["Calls"], "%.3f ms" % (float(x["TotalDurationNs"]) / 1e6), "avg %.1f us" % (float(x["AverageNs"]) / 1e3), x["Percentage"])
PY
