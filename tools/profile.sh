#!/bin/bash
# rocprofv3 evidence for the bench's dominant kernel (run on the GPU box via gpurun).
#   pass 1: kernel trace + stats;  pass 2: FETCH_SIZE;  pass 3: WRITE_SIZE;  pass 4: MFMA busy + clock
#   (separate PMC passes)
# then tools/traffic.py turns them into profiles/<tag>_traffic.json (read by bench.py).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r01}
ARGS=${BENCH_ARGS:-"--steps 10 --warmup 3 --no-extras --no-c3-sharded --no-c5 --no-cpu-baseline"}
X=${PROFILE_EXTRA:-}  # appended to every pass (e.g. --gallery-total 0: the gallery_shard launches only)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" $ARGS $X > "$OUT/bench_trace.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-extras --no-c3-sharded --no-c5 --no-cpu-baseline $X > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-extras --no-c3-sharded --no-c5 --no-cpu-baseline $X > "$OUT/bench_write.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d "$OUT/mfma" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-extras --no-c3-sharded --no-c5 --no-cpu-baseline $X > "$OUT/bench_mfma.log" 2>&1
python3 "$R/tools/traffic.py" "$OUT" "$TAG" > "$OUT/traffic.log" 2>&1
echo "profile done: $OUT"
