#!/bin/bash
# round 6 tree: every -m gpu test, smoke(), and the default bench line -> gpurun_out/${OUT:-final6}/
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=gpurun_out/${OUT:-final6}
cd "$R" && mkdir -p $O || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
d = json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value %.4g' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'frac %.3f' % d['roofline']['frac'], d['roofline']['per_step_check'])
print('b2b %.4f single %.4f' % (d['single_eval_back_to_back_ms'], d['single_eval_ms']), 'cpu', d['cpu_baseline']['value'])
print('c4', json.dumps(d.get('c4_multifusion', {}).get('end_to_end')), 'gallery', d['gallery_shard']['value'])
print('1m', json.dumps({k: d['gallery_1m'].get(k) for k in ('value', 'ms_per_step', 'sampled_rank_mismatches_vs_fp64')}))
print('summary', json.dumps(d.get('summary')))
"
