#!/bin/bash
# K14 evaluation study: eval_bench (events) + a rocprofv3 kernel trace of the same loop.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out || exit 1
timeout -k 10 120 python tools/eval_bench.py ${EVAL_ARGS:-} || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_eval -o run -- python3 $GRAFT_REPO_ROOT/tools/eval_bench.py --reps 100 ${EVAL_ARGS:-} > /dev/null 2>&1 || exit 1
f=$(find $GRAFT_REPO_ROOT/gpurun_out/prof_eval -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -20
