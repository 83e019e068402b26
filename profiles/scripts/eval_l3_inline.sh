#!/bin/bash
# study: level-3 pairs re-scored inside the rank GEMM vs listed for the finish (run at the time as a knob
# CMVE_EVAL_L3_INLINE=1; since adopted for single evaluations: CMVE_EVAL_L3_LIST=1 now selects the list form)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/eval_l3_inline || exit 1
O=gpurun_out/eval_l3_inline
timeout -k 10 600 python -u -m pytest tests/test_gpu_retrieval.py -x -q --timeout 300 --timeout-method thread -k "(level or batch or c1 or dense) and not level3_list" > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
A="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline"
for cfg in "l3list|0" "l3inl|1" "l3list2|0" "l3inl2|1"; do
  n=${cfg%%|*}; v=${cfg#*|}
  CMVE_EVAL_L3_LIST=$((1 - v)) timeout -k 10 200 python bench.py $A > $O/b_$n.json 2> $O/b_$n.err || { echo "$n failed"; tail -5 $O/b_$n.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/b_$n.json').read().strip().splitlines()[-1])
print('$n', 'value %.4g' % d['value'], 'b2b %.4f single %.4f' % (d['single_eval_back_to_back_ms'], d['single_eval_ms']), 'parity', d['recall']['parity_exact'], 'iso', {k: round(v*1e3,1) for k,v in d['kernel_ms_isolated'].items()})
"
done
