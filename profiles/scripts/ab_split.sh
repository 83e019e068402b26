#!/bin/bash
# round 4: the headline with the batches' preps on their own CUs (--cu-split N) vs every launch on every CU
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/split || exit 1
A="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-replay"
for r in 1 2; do
  for n in ${SPLITS:-0 96 112 128}; do
    timeout -k 10 150 python bench.py $A --cu-split $n ${SPLIT_ARGS:-} > gpurun_out/split/s$n.log 2>&1 || { echo "split $n failed"; tail -5 gpurun_out/split/s$n.log; exit 1; }
    python3 -c "
import json; d = json.loads(open('gpurun_out/split/s$n.log').read().strip().splitlines()[-1])
k = d.get('kernel_ms_isolated_batch') or {}
print('split $n: %.4g' % d['value'], 'parity', d['recall']['parity_exact'], 'iso', {a: round(b * 1e3, 1) for a, b in k.items()}, 'inflight', {a: round(b * 1e3, 1) for a, b in d['kernel_ms_inflight'].items()})"
  done
done
