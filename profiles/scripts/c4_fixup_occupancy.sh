#!/bin/bash
# fix-up walk: dynamic LDS prefix + LIGHT dot + occupancy-sized grid; tests, C4 variants, gallery_shard
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/c4_fixup_occupancy || exit 1
O=gpurun_out/c4_fixup_occupancy
timeout -k 10 700 python -u -m pytest tests/test_gpu_fixup_tiled.py tests/test_gpu_retrieval.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
for cfg in "p|-1|0|0" "p_pf|-1|1|0" "t|0|0|0" "t_pf|0|1|0" "p_b128|-1|0|128" "t2|2|0|0"; do
  IFS='|' read n g pf bpx <<< "$cfg"
  CMVE_CIRR_FIX_GROUP=$g CMVE_FIX_PF=$pf CMVE_FIX_BPX=$bpx timeout -k 10 240 python tools/fusion_bench.py --loop-q 0 --sample 64 > $O/c4_$n.json 2> $O/c4_$n.err || { echo "c4 $n failed"; tail -5 $O/c4_$n.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c4_$n.json').read().strip().splitlines()[-1])
r=d['ranking']; print('$n', 'rank ms %.2f' % r['ms'], 'mism', r['fp64_sample']['mismatches'], 'R1 %.4f' % r['recall_at_1_5_10_50'][0])
"
done
A="--steps 2 --warmup 1 --evals-per-step 8 --no-extras --no-cpu-baseline --no-replay --no-c3-sharded --no-c5"
for cfg in "s|0|0" "s_pf|1|0" "s_b128|0|128"; do
  IFS='|' read n pf bpx <<< "$cfg"
  CMVE_FIX_PF=$pf CMVE_FIX_BPX=$bpx timeout -k 10 300 python bench.py $A > $O/b_$n.json 2> $O/b_$n.err || { echo "$n failed"; tail -5 $O/b_$n.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/b_$n.json').read().strip().splitlines()[-1])
g=d['gallery_shard']; m=d.get('gallery_1m', {})
print('$n', 'shard rank ms %.3f fix ms %.3f' % (g['rank_count']['ms'], g['rank_count']['fixup_ms']), 'v %.4g' % g['value'], '1m', m.get('value'), (m.get('rank_count') or {}).get('fixup_ms'))
"
done
