#!/bin/bash
# chained batch runs + tiled fix-up: tests, C4 ranking A/B over the fix-up grouping, headline A/B
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/ab_chain_tiled || exit 1
O=gpurun_out/ab_chain_tiled
timeout -k 10 600 python -u -m pytest tests/test_gpu_fixup_tiled.py tests/test_gpu_batch_checks.py tests/test_gpu_retrieval.py -k "tiled or batch or chained or unaligned or paired_flag or cu_mask" -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
for gset in -1 0 1 2 4 -1b 0b; do
  g=${gset%b}
  CMVE_CIRR_FIX_GROUP=$g timeout -k 10 240 python tools/fusion_bench.py --loop-q 0 --sample 64 > $O/c4_$gset.json 2> $O/c4_$gset.err || { echo "c4 $gset failed"; tail -5 $O/c4_$gset.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c4_$gset.json').read().strip().splitlines()[-1])
r=d['ranking']; print('group $gset', 'rank ms %.2f' % r['ms'], 'mism', r['fp64_sample']['mismatches'], 'R', r['recall_at_1_5_10_50'], 'e2e q/s %.3g' % d['end_to_end']['queries_per_s'])
"
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/c4k -o run -- python3 "$R/tools/fusion_bench.py" --loop-q 0 --sample 16 > "$R/$O/c4k.log" 2>&1 || { tail -5 "$R/$O/c4k.log"; exit 1; }
f=$(find /tmp/c4k -name "*kernel_stats.csv" | head -1); cp "$f" "$R/$O/c4_kernel_stats.csv"
python3 - "$R/$O/c4_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("fixup", "tile_sort", "sim_kernel", "gt_thr", "cand_final")):
        print(n[:60], r["Calls"], "avg ms %.3f" % (float(r["AverageNs"]) / 1e6), "tot ms %.2f" % (float(r["TotalDurationNs"]) / 1e6))
PY
cd "$R"
A="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-replay"
for cfg in "c1|--chain 1" "c0|--chain 0" "c1b|--chain 1" "c0b|--chain 0" "c1s4|--chain 1 --inflight 4" "c1s2|--chain 1 --inflight 2"; do
  n=${cfg%%|*}; f=${cfg#*|}
  timeout -k 10 200 python bench.py $A $f > $O/b_$n.json 2> $O/b_$n.err || { echo "$n failed"; tail -5 $O/b_$n.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$O/b_$n.json').read().strip().splitlines()[-1])
print('$n', 'value %.4g' % d['value'], 'parity', d['recall']['parity_exact'], 'inflight', {k: round(v*1e3,1) for k,v in d['kernel_ms_inflight'].items()})
"
done
