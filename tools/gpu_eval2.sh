#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_retrieval.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
grep -E "^E |Error|assert" gpurun_out/t.log | head -20
bash tools/gpu_eval.sh
