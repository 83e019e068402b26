#!/bin/bash
# round 6: rocprofv3 evidence for the gallery_1m leg (16,384 x 1,048,576 x 1024 in 8 chunks of 131,072 rows, each
# chunk's fix-up overlapped with the next chunk's MFMA pass): kernel trace + stats, FETCH_SIZE, WRITE_SIZE, MFMA busy
# -> profiles/r06_g1m_traffic.json + r06_g1m_kernel_stats.csv (bench.py --traffic-g1m-json default)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" || exit 1
export BENCH_ARGS="--steps 3 --warmup 1 --no-extras --no-c3-sharded --no-c5 --no-cpu-baseline"
export PROFILE_EXTRA="--no-gallery-shard --no-replay --shard-steps 5"
export SHARD=1048576 CHUNKS=8 TRACE_TIMED_STEPS=40
bash tools/profile.sh r06_g1m && cp gpurun_out/prof_r06_g1m/profiles/* profiles/ 2>/dev/null; \
  cat gpurun_out/prof_r06_g1m/traffic.log | tail -2
