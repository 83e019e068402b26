#!/bin/bash
# C4 (MultiFusion composed path) parity + bench (+ optional rocprofv3 kernel stats) on the GPU box.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
timeout -k 10 300 python -u -m pytest tests/test_combiner.py tests/test_multifusion_rank.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/c4_tests.log 2>&1 \
  && timeout -k 10 300 python tools/fusion_bench.py > gpurun_out/fusion_bench.log 2>&1
rc=$?
echo "rc=$rc"; tail -5 gpurun_out/c4_tests.log; tail -1 gpurun_out/fusion_bench.log
if [ $rc -eq 0 ] && [ -n "$C4_PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_c4" -o run -- python3 "$R/tools/fusion_bench.py" --nq 8192 --loop-q 32 > "$R/gpurun_out/prof_c4.log" 2>&1
  rc=$?
  echo "prof rc=$rc"
fi
exit $rc
