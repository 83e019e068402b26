#!/bin/bash
# 1k-A headline: one evaluation per launch set (3 streams) vs K-evaluation batches (cmve_eval_batch_*), alternating
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
ARGS="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-c3-sharded --no-c5"
VARIANTS=${AB_VARIANTS:-"base:--batch=1 b10:--batch=10 b20:--batch=20 b10s2:--batch=10,--inflight=2 b5s4:--batch=5,--inflight=4"}
for r in 1 2; do
  for v in $VARIANTS; do
    name=${v%%:*}; extra=${v#*:}; extra=${extra//,/ }
    timeout -k 10 120 python bench.py $ARGS $extra > gpurun_out/abb_${name}_$r.log 2>&1 || exit 1
    echo "$name $r: $(grep -o '"value": [0-9.e+]*' gpurun_out/abb_${name}_$r.log | head -1) $(grep -o '"single_set_replay": {"value": [0-9.e+]*' gpurun_out/abb_${name}_$r.log) $(grep -o '"parity_exact": [a-z]*' gpurun_out/abb_${name}_$r.log)"
  done
done
