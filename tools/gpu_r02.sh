#!/bin/bash
# Round-2 GPU check: the changed areas first (NaN ranks, K14 evaluation, sharded merge), then the
# full GPU suite, smoke() and the default bench line.  Each GPU step has its own time limit.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_retrieval.py -x -v --timeout 120 --timeout-method thread -k "nan or session or shards or sharded" > gpurun_out/gpu_new.log 2>&1 \
  && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  && timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?
echo "rc=$rc"
tail -3 gpurun_out/gpu_new.log; grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -3
tail -1 gpurun_out/smoke.log 2>/dev/null
tail -c 1500 gpurun_out/bench.log 2>/dev/null
exit $rc
