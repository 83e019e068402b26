#!/bin/bash
# C4 fix-up study: tiled grouping x GT-score prefetch x blocks per XCD, then FETCH_SIZE of plain vs tiled
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/c4_fixup_study || exit 1
O=gpurun_out/c4_fixup_study
timeout -k 10 300 python -u -m pytest tests/test_gpu_fixup_tiled.py -x -q --timeout 150 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
for cfg in "p|-1|0|128" "t|0|0|128" "p_pf|-1|1|128" "t_pf|0|1|128" "p_b256|-1|0|256" "t_pf_b256|0|1|256" "t2_pf|2|1|128" "p_pf_b64|-1|1|64"; do
  IFS='|' read n g pf bpx <<< "$cfg"
  CMVE_CIRR_FIX_GROUP=$g CMVE_FIX_PF=$pf CMVE_FIX_BPX=$bpx timeout -k 10 240 python tools/fusion_bench.py --loop-q 0 --sample 64 > $O/c4_$n.json 2> $O/c4_$n.err || { echo "c4 $n failed"; tail -5 $O/c4_$n.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c4_$n.json').read().strip().splitlines()[-1])
r=d['ranking']; print('$n', 'rank ms %.2f' % r['ms'], 'mism', r['fp64_sample']['mismatches'], 'R1 %.4f' % r['recall_at_1_5_10_50'][0])
"
done
cd /tmp && export TMPDIR=/tmp
for g in -1 0; do
  CMVE_CIRR_FIX_GROUP=$g timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/fx$g -o run -- python3 "$R/tools/fusion_bench.py" --loop-q 0 --sample 16 > "$R/$O/fetch$g.log" 2>&1 || { tail -5 "$R/$O/fetch$g.log"; exit 1; }
  python3 - /tmp/fx$g $g <<'PY'
import collections, csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if r["Counter_Name"] == "FETCH_SIZE":
        d[r["Kernel_Name"][:40]].append((float(r["Counter_Value"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
for k, v in d.items():
    if "fixup" in k or "tile_sort" in k:
        for x in v[-2:]:
            print("group", sys.argv[2], k, "fetched GB %.2f" % (2 * x[0] * 1024 / 1e9), "ms %.3f" % x[1])
PY
done
