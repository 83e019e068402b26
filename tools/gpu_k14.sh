#!/bin/bash
# K14 check: the evaluation's GPU tests, then eval_bench (events) and a rocprofv3 kernel trace of it.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_retrieval.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k14_tests.log 2>&1
rc=$?; tail -2 gpurun_out/k14_tests.log; grep -E "^E |Error" gpurun_out/k14_tests.log | head -10
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_eval.sh
