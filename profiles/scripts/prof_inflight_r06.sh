#!/bin/bash
# round 6: kernel trace of the headline with its three batches in flight (the default line's loop) ->
# gpurun_out/r06_inflight/, reduced by tools/inflight_timeline.py
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06_inflight
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-shard-leg --no-extras --no-cpu-baseline --no-replay --steps 20 --warmup 2 > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
f=$(find $O/trace -name "run_kernel_trace.csv" | head -1)
python3 $R/tools/inflight_timeline.py $f | tee $O/timeline.txt
