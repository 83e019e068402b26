#!/bin/bash
# Run the named GPU test files (default: the ones changed this session), each step time-limited.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
FILES=${TEST_FILES:-"tests/test_dual.py tests/test_multifusion_infer.py tests/test_abi.py"}
timeout -k 10 400 python -u -m pytest $FILES -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_new.log 2>&1
rc=$?
tail -25 gpurun_out/gpu_new.log
exit $rc
