#!/bin/bash
# PMC pass over the kernel micro-bench (run on the GPU box via gpurun): effective clock
# (GRBM_GUI_ACTIVE / 8 / duration) and MFMA busy cycles of the sim kernels.  Counter runs use
# --kernel-trace only (no runtime/sys trace domains).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-pmc}
COUNTERS=${COUNTERS:-"GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc $COUNTERS --kernel-trace --output-format csv -d "$OUT" -o run -- python3 "$R/tools/kbench.py" > "$OUT/kbench.log" 2>&1
echo "pmc done: $OUT"
