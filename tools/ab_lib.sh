#!/bin/bash
# A/B of the 1k-A headline: the product library vs a study library (AB_LIB), alternating, same box
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
ARGS="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-c3-sharded --no-c5 ${AB_ARGS:-}"
for r in 1 2; do
  timeout -k 10 100 python bench.py $ARGS > gpurun_out/ab_base_$r.log 2>&1 || exit 1
  env CMVE_LIB=$R/$AB_LIB ${AB_ENV:-} timeout -k 10 100 python bench.py $ARGS > gpurun_out/ab_alt_$r.log 2>&1 || exit 1
  for k in base alt; do
    echo "$k $r: $(grep -o '"value": [0-9.e+]*' gpurun_out/ab_${k}_$r.log | head -1) $(grep -o '"single_set_replay": {"value": [0-9.e+]*' gpurun_out/ab_${k}_$r.log) $(grep -o '"single_eval_back_to_back_ms": [0-9.e+-]*' gpurun_out/ab_${k}_$r.log) $(grep -o '"parity_exact": [a-z]*' gpurun_out/ab_${k}_$r.log)"
  done
done
