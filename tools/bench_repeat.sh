#!/bin/bash
# the default bench line's headline, REPS times in fresh processes, driver-style (--steps 20): run-to-run spread
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
for r in $(seq 1 ${REPS:-6}); do
  timeout -k 10 100 python bench.py --steps ${STEPS:-20} --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-c3-sharded --no-c5 ${BENCH_ARGS:-} > gpurun_out/rep_$r.log 2>&1 || exit 1
  echo "$r: $(grep -o '"value": [0-9.e+]*' gpurun_out/rep_$r.log | head -1) $(grep -o '"ms_per_step": [0-9.e+]*' gpurun_out/rep_$r.log | head -1)"
done
