#!/bin/bash
# A/B of the 1k-A headline: the product library vs several study libraries (AB_LIBS="name:path ..."), alternating
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
ARGS="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-c3-sharded --no-c5 ${AB_ARGS:-}"
for r in 1 2; do
  timeout -k 10 100 python bench.py $ARGS > gpurun_out/abl_base_$r.log 2>&1 || exit 1
  echo "base $r: $(grep -o '"value": [0-9.e+]*' gpurun_out/abl_base_$r.log | head -1) $(grep -o '"single_eval_back_to_back_ms": [0-9.e+-]*' gpurun_out/abl_base_$r.log) $(grep -o '"parity_exact": [a-z]*' gpurun_out/abl_base_$r.log)"
  for v in $AB_LIBS; do
    n=${v%%:*}; l=${v#*:}
    CMVE_LIB=$R/$l timeout -k 10 100 python bench.py $ARGS > gpurun_out/abl_${n}_$r.log 2>&1 || exit 1
    echo "$n $r: $(grep -o '"value": [0-9.e+]*' gpurun_out/abl_${n}_$r.log | head -1) $(grep -o '"single_eval_back_to_back_ms": [0-9.e+-]*' gpurun_out/abl_${n}_$r.log) $(grep -o '"parity_exact": [a-z]*' gpurun_out/abl_${n}_$r.log)"
  done
done
