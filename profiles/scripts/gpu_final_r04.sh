#!/bin/bash
# round 4 final tree: every -m gpu test, smoke(), and the default bench line -> gpurun_out/final/
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/final || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/final/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.txt 2>&1 || { tail -5 gpurun_out/final/smoke.txt; exit 1; }
tail -1 gpurun_out/final/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/final/bench.json').read().strip().splitlines()[-1])
print('value %.4g' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'frac %.3f' % d['roofline']['frac'], d['roofline']['per_step_check'])
print('b2b %.4f single %.4f' % (d['single_eval_back_to_back_ms'], d['single_eval_ms']), 'cpu', d['cpu_baseline']['value'])
print('c4', json.dumps(d.get('c4_multifusion', {}).get('end_to_end')), 'gallery', d['gallery_shard']['value'])
"
