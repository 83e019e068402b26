#!/bin/bash
# Round-3 GPU check: the full GPU suite, smoke() and the default bench line (the driver's own
# commands), then (PROFILE=tag) the rocprofv3 evidence of the headline.  Each GPU step has its own
# time limit and the steps are chained, so the first failure ends the call.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  && timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?
echo "rc=$rc"
grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -3
tail -1 gpurun_out/smoke.log 2>/dev/null
tail -c 2500 gpurun_out/bench.log 2>/dev/null
if [ $rc -eq 0 ] && [ -n "${PROFILE:-}" ]; then
  bash "$R/tools/profile_1ka.sh" "$PROFILE"
  rc=$?
  tail -5 "$R/gpurun_out/prof1ka_$PROFILE/traffic.log"
fi
exit $rc
