#!/bin/bash
# 1k-A single-set replay: direct launches vs captured HIP graphs (host cost per evaluation), alternating
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
ARGS="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-c3-sharded --no-c5 --input-sets 1"
for r in 1 2; do
  timeout -k 10 100 python bench.py $ARGS > gpurun_out/abg_direct_$r.log 2>&1 || exit 1
  timeout -k 10 100 python bench.py $ARGS --graphs > gpurun_out/abg_graphs_$r.log 2>&1 || exit 1
  for k in direct graphs; do
    echo "$k $r: $(grep -o '"value": [0-9.e+]*' gpurun_out/abg_${k}_$r.log | head -1) $(grep -o '"parity_exact": [a-z]*' gpurun_out/abg_${k}_$r.log)"
  done
done
