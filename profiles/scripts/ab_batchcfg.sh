#!/bin/bash
# round 4: the headline over batch sizes / streams in flight (the kernels changed since round 3's sweep)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/bcfg || exit 1
A="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-replay"
for r in 1 2; do
  for cfg in ${CFGS:-"8 3 24" "8 2 24" "8 4 24" "12 3 24" "12 2 24" "6 3 24" "16 2 32"}; do
    set -- $cfg
    timeout -k 10 150 python bench.py $A --batch $1 --inflight $2 --input-sets $3 > gpurun_out/bcfg/b$1_$2.log 2>&1 || { echo "cfg $cfg failed"; tail -3 gpurun_out/bcfg/b$1_$2.log; continue; }
    echo "batch $1 inflight $2 sets $3: $(grep -o '"value": [0-9.e+]*' gpurun_out/bcfg/b$1_$2.log | head -1)"
  done
done
