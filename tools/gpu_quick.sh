#!/bin/bash
# quick GPU iteration: the named pytest files (TESTS), then a short bench line (BENCH_ARGS); each step
# under its own time limit, chained so that the first failure ends the call.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
timeout -k 10 ${TEST_LIMIT:-500} python -u -m pytest ${TESTS:-tests -m gpu} -x -v --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|error|Error" gpurun_out/quick_tests.log | tail -5
[ $rc -ne 0 ] && exit $rc
if [ -n "${BENCH_ARGS+x}" ]; then
  timeout -k 10 ${BENCH_LIMIT:-400} python bench.py $BENCH_ARGS > gpurun_out/quick_bench.log 2>&1
  rc=$?
  echo "bench rc=$rc"; tail -c 3000 gpurun_out/quick_bench.log
fi
exit $rc
