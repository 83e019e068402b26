#!/bin/bash
# single evaluations re-score their level-3 pairs in the rank GEMM (default) vs the list form (CMVE_EVAL_L3_LIST=1)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/eval_l3_single || exit 1
O=gpurun_out/eval_l3_single
timeout -k 10 700 python -u -m pytest tests/test_gpu_retrieval.py tests/test_gpu_batch_checks.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
A="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline"
for cfg in "inl|0" "list|1" "inl2|0" "list2|1"; do
  n=${cfg%%|*}; v=${cfg#*|}
  CMVE_EVAL_L3_LIST=$v timeout -k 10 200 python bench.py $A > $O/b_$n.json 2> $O/b_$n.err || { echo "$n failed"; tail -5 $O/b_$n.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/b_$n.json').read().strip().splitlines()[-1])
print('$n', 'value %.4g b2b %.4f graph b2b %s' % (d['value'], d['single_eval_back_to_back_ms'], d.get('single_eval_graph_back_to_back_ms')), 'parity', d['recall']['parity_exact'], 'iso', {k: round(v*1e3,1) for k,v in d['kernel_ms_isolated'].items()})
"
done
