#!/bin/bash
# full GPU parity suite + smoke + C4 bench (after a kernel change)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  && timeout -k 10 300 python tools/fusion_bench.py > gpurun_out/fusion_bench.log 2>&1
rc=$?
echo "rc=$rc"
grep -E "passed|failed|error|FAIL" gpurun_out/gpu_tests.log | tail -5
tail -1 gpurun_out/smoke.log; tail -1 gpurun_out/fusion_bench.log
exit $rc
