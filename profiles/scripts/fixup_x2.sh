#!/bin/bash
# study: two pairs per wave in the fix-up walk (CMVE_FIX_X2=1), C4 ranking + gallery shard / 1M fix-ups
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/fixup_x2 || exit 1
O=gpurun_out/fixup_x2
CMVE_FIX_X2=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fixup_tiled.py tests/test_gpu_retrieval.py -x -q --timeout 300 --timeout-method thread -k "tiled or fused or overlap or bench_shape or c3 or nan or topk" > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
for cfg in "x1|0" "x2|1" "x1b|0" "x2b|1"; do
  n=${cfg%%|*}; v=${cfg#*|}
  CMVE_FIX_X2=$v timeout -k 10 240 python tools/fusion_bench.py --loop-q 0 --sample 64 > $O/c4_$n.json 2> $O/c4_$n.err || { echo "c4 $n failed"; tail -5 $O/c4_$n.err; exit 1; }
  CMVE_FIX_X2=$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --evals-per-step 8 --no-extras --no-cpu-baseline --no-replay --no-c3-sharded --no-c5 --g1m-chunks 1 > $O/b_$n.json 2> $O/b_$n.err || { echo "b $n failed"; tail -5 $O/b_$n.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c4_$n.json').read().strip().splitlines()[-1]); r=d['ranking']
b=json.loads(open('$O/b_$n.json').read().strip().splitlines()[-1]); g=b['gallery_shard']; m=b['gallery_1m']
print('$n', 'c4 rank ms %.2f mism %d' % (r['ms'], r['fp64_sample']['mismatches']), '| shard fix ms %.3f v %.4g' % (g['rank_count']['fixup_ms'], g['value']), '| 1m fix ms %.2f v %.4g mism %s' % (m['rank_count']['fixup_ms'], m['value'], m['sampled_rank_mismatches_vs_fp64']))
"
done
