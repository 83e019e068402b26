#!/bin/bash
# headline batch / stream sweep on the chained round-5 kernels (two passes)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/ab_batchcfg_r05 || exit 1
O=gpurun_out/ab_batchcfg_r05
A="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-replay"
for pass in 1 2; do
for cfg in "b8s3|--batch 8 --inflight 3" "b12s3|--batch 12 --inflight 3 --input-sets 24" "b16s2|--batch 16 --inflight 2 --input-sets 32" "b8s2|--batch 8 --inflight 2" "b10s3|--batch 10 --inflight 3 --input-sets 30" "b6s4|--batch 6 --inflight 4"; do
  n=${cfg%%|*}; f=${cfg#*|}
  timeout -k 10 200 python bench.py $A $f > $O/b_${n}_$pass.json 2> $O/b_${n}_$pass.err || { echo "$n failed"; tail -5 $O/b_${n}_$pass.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/b_${n}_$pass.json').read().strip().splitlines()[-1])
print('$n $pass', 'value %.4g' % d['value'], 'parity', d['recall']['parity_exact'])
"
done
done
