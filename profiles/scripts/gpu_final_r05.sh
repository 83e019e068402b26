#!/bin/bash
# round 5 final tree: every -m gpu test, smoke(), and the default bench line -> gpurun_out/final5/
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/final5 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final5/gpu_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/final5/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final5/smoke.txt 2>&1 || { tail -5 gpurun_out/final5/smoke.txt; exit 1; }
tail -1 gpurun_out/final5/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/final5/bench.json 2> gpurun_out/final5/bench.err || { tail -20 gpurun_out/final5/bench.err; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/final5/bench.json').read().strip().splitlines()[-1])
print('value %.4g' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'frac %.3f' % d['roofline']['frac'], d['roofline']['per_step_check'])
print('b2b %.4f single %.4f' % (d['single_eval_back_to_back_ms'], d['single_eval_ms']), 'cpu', d['cpu_baseline']['value'])
print('c4', json.dumps(d.get('c4_multifusion', {}).get('end_to_end')), 'gallery', d['gallery_shard']['value'])
"
python3 -c "
import json
d = json.loads(open('gpurun_out/final5/bench.json').read().strip().splitlines()[-1])
print('1m', json.dumps({k: d['gallery_1m'].get(k) for k in ('value', 'ms_per_step', 'sampled_rank_mismatches_vs_fp64')}))
print('c4 ranking', json.dumps(d.get('c4_multifusion', {}).get('ranking')))
"
