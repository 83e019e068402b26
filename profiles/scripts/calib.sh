#!/bin/bash
# rocprofv3 counter calibration (run on the GPU box via gpurun): tools/calib.py's known-byte launches under a
# FETCH_SIZE pass and a WRITE_SIZE pass (each with --kernel-trace only), reduced by tools/calib_reduce.py.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
OUT=$R/gpurun_out/calib
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- python3 "$R/tools/calib.py" "$OUT" > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- python3 "$R/tools/calib.py" "$OUT" > "$OUT/write.log" 2>&1
python3 "$R/tools/calib_reduce.py" "$OUT"
