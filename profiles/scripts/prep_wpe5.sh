#!/bin/bash
# study: the paired prep at 5 waves per SIMD (<= 96 VGPRs, 8 spilled) vs 4
# (scratch/libcmve_pw5.so: eval.hip rebuilt with -DCMVE_PREPFIN_WPE=5 -DCMVE_PREP_WPE=5 and linked with the other objects)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/prep_wpe5 || exit 1
O=gpurun_out/prep_wpe5
A="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-replay"
for cfg in "w4|" "w5|$R/scratch/libcmve_pw5.so" "w4b|" "w5b|$R/scratch/libcmve_pw5.so"; do
  n=${cfg%%|*}; lib=${cfg#*|}
  if [ -n "$lib" ]; then export CMVE_LIB=$lib; else unset CMVE_LIB; fi
  timeout -k 10 200 python bench.py $A > $O/b_$n.json 2> $O/b_$n.err || { echo "$n failed"; tail -5 $O/b_$n.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/b_$n.json').read().strip().splitlines()[-1])
print('$n', 'value %.4g' % d['value'], 'parity', d['recall']['parity_exact'], 'iso batch', {k: round(v*1e3,1) for k,v in d['kernel_ms_isolated_batch'].items()}, 'b2b %.4f' % d['single_eval_back_to_back_ms'])
"
done
