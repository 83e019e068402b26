#!/bin/bash
# fix-up study: parity, then A/B of the fix-up time (tools/ab.sh with the fix-up timed)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
L=$R/cross-modal-video-engine_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_retrieval.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fix_tests.log 2>&1 || { tail -20 gpurun_out/fix_tests.log; exit 1; }
tail -1 gpurun_out/fix_tests.log
AB_NOFIX= A=$L/diag/libcmve_base.so B=$L/cmve/libcmve.so timeout -k 10 600 bash tools/ab.sh
