#!/bin/bash
# round 4: C4 end to end (30,364 queries, no per-batch loop) for mha_absorbed variants: CMVE_MHA_HPW x CMVE_MHA_ROWS
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/abm || exit 1
for v in ${MHA_VARS:-"4 1" "2 1" "2 2" "2 4" "4 2"}; do
  set -- $v
  CMVE_MHA_HPW=$1 CMVE_MHA_ROWS=$2 timeout -k 10 200 python3 tools/fusion_bench.py --loop-q 0 --sample 64 > gpurun_out/abm/h$1r$2.json 2> gpurun_out/abm/h$1r$2.err || { tail -5 gpurun_out/abm/h$1r$2.err; exit 1; }
  python3 - gpurun_out/abm/h$1r$2.json "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print("hpw/rows", sys.argv[2], "combine %.1f ms %.4g q/s" % (d["combine_batches"]["ms"], d["combine_batches"]["queries_per_s"]),
      "rank %.1f ms" % d["ranking"]["ms"], "mism", d["ranking"]["fp64_sample"]["mismatches"])
PY
done
