#!/bin/bash
# rocprofv3 kernel trace + stats of one python tool: bash tools/gpu_prof_one.sh TAG tools/x.py [args]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/$@" > "$R/gpurun_out/prof_$TAG.log" 2>&1
rc=$?
echo "rc=$rc"; tail -2 "$R/gpurun_out/prof_$TAG.log"
exit $rc
