#!/bin/bash
# Round-2 refresh: full GPU suite, smoke(), rocprofv3 evidence of the 1k-A headline (r02d) and of the
# gallery_shard rank kernel, the default bench line, the fp8 band study.  Each GPU step has its own limit.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  && bash tools/profile_1ka.sh ${TAG:-r02d} > gpurun_out/prof1ka.log 2>&1 \
  && cp gpurun_out/prof1ka_${TAG:-r02d}/profiles/${TAG:-r02d}_1ka_traffic.json profiles/ \
  && BENCH_ARGS="--steps 200 --warmup 5 --no-extras --no-cpu-baseline --no-c3-sharded --shard-steps 10" bash tools/profile.sh ${TAG:-r02d} > gpurun_out/prof_shard.log 2>&1 \
  && cp gpurun_out/prof_${TAG:-r02d}/profiles/${TAG:-r02d}_traffic.json profiles/ \
  && cd "$R" && timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 \
  && timeout -k 10 200 python tools/fp8_study.py > gpurun_out/fp8.log 2>&1
rc=$?
echo "rc=$rc"
grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -3
tail -1 gpurun_out/smoke.log 2>/dev/null
tail -c 600 gpurun_out/bench.log 2>/dev/null
exit $rc
