#!/bin/bash
# K14 batches: rank-GEMM geometry x batch size, alternating (CMVE_BATCH_GEO: default 128 x 64, 128128 = 8-wave 128 x 128)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
A="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-c3-sharded --no-c5"
V=${GEO_VARIANTS:-"b10::--batch=10 g128b10:CMVE_BATCH_GEO=128128:--batch=10"}
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in $V; do
    n=${v%%:*}; rest=${v#*:}; e=${rest%%:*}; a=${rest#*:}; a=${a//,/ }; a=${a//=/ }
    env $e timeout -k 10 120 python bench.py $A $a > gpurun_out/g_$n.log 2>&1 || exit 1
    echo "$n $r: $(grep -o '"value": [0-9.e+]*' gpurun_out/g_$n.log | head -1) $(grep -o '"parity_exact": [a-z]*' gpurun_out/g_$n.log | head -1)"
  done
done
