#!/bin/bash
# 1k-A headline: hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4) x evaluations in flight
# (kernel studies; each run its own process, --steps 20 as the driver runs it)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
for q in ${SWEEP_Q:-4 8}; do for n in ${SWEEP_N:-3 4 6 8}; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-shard-leg --no-extras \
    --no-cpu-baseline --no-c3-sharded --no-c5 --inflight $n > gpurun_out/qs_${q}_${n}.log 2>&1 || exit 1
  echo "queues $q inflight $n: $(grep -o '"value": [0-9.e+]*' gpurun_out/qs_${q}_${n}.log | head -1)"
done; done
