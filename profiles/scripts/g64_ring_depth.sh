#!/bin/bash
# study: deeper G64 ring (single-evaluation rank GEMM) x level-3 inline, single-evaluation latency
# (libcmve_g64s{6,8}.so: sim.hip rebuilt with -DCMVE_G64_STAGES=6 / 8 and linked with the other objects under scratch/)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/g64_ring_depth || exit 1
O=gpurun_out/g64_ring_depth
A="--steps 4 --warmup 2 --no-shard-leg --no-extras --no-cpu-baseline --no-replay"
for cfg in "s4|0|" "s6|0|$R/scratch/libcmve_g64s6.so" "s8|0|$R/scratch/libcmve_g64s8.so" "s8i|1|$R/scratch/libcmve_g64s8.so" "s4i|1|" "s8b|0|$R/scratch/libcmve_g64s8.so" "s4b|0|"; do
  IFS='|' read n inl lib <<< "$cfg"
  if [ -n "$lib" ]; then export CMVE_LIB=$lib; else unset CMVE_LIB; fi
  CMVE_EVAL_L3_LIST=$((1 - inl)) timeout -k 10 200 python bench.py $A > $O/b_$n.json 2> $O/b_$n.err || { echo "$n failed"; tail -5 $O/b_$n.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/b_$n.json').read().strip().splitlines()[-1])
print('$n', 'b2b %.4f single %.4f' % (d['single_eval_back_to_back_ms'], d['single_eval_ms']), 'parity', d['recall']['parity_exact'], 'iso', {k: round(v*1e3,1) for k,v in d['kernel_ms_isolated'].items()})
"
done
