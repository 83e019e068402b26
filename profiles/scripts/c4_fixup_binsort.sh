#!/bin/bash
# tiled fix-up v2: pairs sorted by query within (super-bucket, tile) bins, walked in per-wave runs
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/c4_fixup_binsort || exit 1
O=gpurun_out/c4_fixup_binsort
timeout -k 10 300 python -u -m pytest tests/test_gpu_fixup_tiled.py -x -q --timeout 150 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
for cfg in "p|-1|16|1" "t|0|16|1" "t_r1|0|1|1" "t_r64|0|64|1" "t_nobin|0|16|0" "t2|2|16|1" "t1|1|16|1" "t4|4|16|1" "p2|-1|16|1"; do
  IFS='|' read n g run bins <<< "$cfg"
  CMVE_CIRR_FIX_GROUP=$g CMVE_FIX_RUN=$run CMVE_FIX_BINSORT=$bins timeout -k 10 240 python tools/fusion_bench.py --loop-q 0 --sample 64 > $O/c4_$n.json 2> $O/c4_$n.err || { echo "c4 $n failed"; tail -5 $O/c4_$n.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c4_$n.json').read().strip().splitlines()[-1])
r=d['ranking']; print('$n', 'rank ms %.2f' % r['ms'], 'mism', r['fp64_sample']['mismatches'], 'R1 %.4f' % r['recall_at_1_5_10_50'][0])
"
done
cd /tmp && export TMPDIR=/tmp
for g in -1 0; do
  CMVE_CIRR_FIX_GROUP=$g timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d /tmp/l2$g -o run -- python3 "$R/tools/fusion_bench.py" --loop-q 0 --sample 16 > "$R/$O/l2$g.log" 2>&1 || { tail -5 "$R/$O/l2$g.log"; exit 1; }
  python3 - /tmp/l2$g $g <<'PY'
import collections, csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:40]
    if "fixup" in k or "tile_sort" in k:
        d[(k, r["Dispatch_Id"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        d[(k, r["Dispatch_Id"])]["ms"] = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6]
for (k, di), v in list(d.items())[-6:]:
    h, m = sum(v["TCC_HIT_sum"]), sum(v["TCC_MISS_sum"])
    print("group", sys.argv[2], k, di, "ms %.3f hit %.3g miss %.3g hit rate %.3f" % (v["ms"][0], h, m, h / max(1, h + m)))
PY
done
