#!/bin/bash
# Round-end style check on the GPU box: GPU parity tests, smoke(), default bench line.
# Each GPU step has its own time limit; the chain stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  && timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?
echo "rc=$rc"
grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -3
tail -1 gpurun_out/smoke.log 2>/dev/null
tail -c 600 gpurun_out/bench.log 2>/dev/null
exit $rc
