#!/bin/bash
# epilogue study: parity of the rank / top-k paths, stamps of the new epilogue, A/B vs the base build
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
L=$R/cross-modal-video-engine_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_retrieval.py tests/test_gpu_topk.py -x -q --timeout 120 --timeout-method thread > gpurun_out/epi_tests.log 2>&1 || { tail -20 gpurun_out/epi_tests.log; exit 1; }
tail -1 gpurun_out/epi_tests.log
KB_STAMPS=real KB_NOFIX=1 CMVE_LIB=$L/diag/libcmve_STAMPS.so MODES=F16 REPS=5 timeout -k 10 200 python tools/kbench.py 2>&1 | grep -E "stamps" || exit 1
A=$L/diag/libcmve_base.so B=$L/cmve/libcmve.so timeout -k 10 600 bash tools/ab.sh
