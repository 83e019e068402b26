#!/bin/bash
# rocprofv3 evidence for the 1k-A headline's three evaluation launches (run on the GPU box via gpurun):
#   pass 1: kernel trace + stats of the headline loop;  pass 2: FETCH_SIZE;  pass 3: WRITE_SIZE
# (separate PMC passes), reduced by tools/traffic_1ka.py into profiles/<tag>_1ka_traffic.json.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r02}
ARGS="--steps 200 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline"
OUT=$R/gpurun_out/prof1ka_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/bench_trace.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "$R/bench.py" --steps 20 --warmup 2 --no-shard-leg --no-extras --no-cpu-baseline > "$OUT/bench_fetch.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "$R/bench.py" --steps 20 --warmup 2 --no-shard-leg --no-extras --no-cpu-baseline > "$OUT/bench_write.log" 2>&1
python3 "$R/tools/traffic_1ka.py" "$OUT" "$TAG" > "$OUT/traffic.log" 2>&1
echo "profile 1ka done: $OUT"
