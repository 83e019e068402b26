#!/bin/bash
# End-of-round check: the full GPU suite, smoke(), the default bench line, and the per-evaluation form of the
# headline (--batch 1 --inflight 3) as a sanity run of the non-batched loop
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  && timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 \
  && timeout -k 10 120 python bench.py --steps 20 --batch 1 --inflight 3 --no-shard-leg --no-extras --no-cpu-baseline --no-c3-sharded --no-c5 > gpurun_out/bench_b1.log 2>&1
rc=$?
echo "rc=$rc"
grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -2
tail -1 gpurun_out/smoke.log 2>/dev/null
for f in bench bench_b1; do echo "$f: $(grep -o '"value": [0-9.e+]*' gpurun_out/$f.log | head -1) $(grep -o '"parity_exact": [a-z]*' gpurun_out/$f.log | head -1)"; done
exit $rc
