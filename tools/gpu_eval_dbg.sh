#!/bin/bash
# K14 kernel study: rocprof kernel times of the evaluation with parts disabled (CMVE_EVAL_DBG bits)
cd /tmp && export TMPDIR=/tmp
for D in 0 1 2 4 3 8 16 32 24; do
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_dbg_$D
  CMVE_EVAL_DBG=$D timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dbg_$D -o run -- python3 $GRAFT_REPO_ROOT/tools/eval_bench.py --reps 100 > /dev/null 2>&1 || exit 1
  f=$(find $GRAFT_REPO_ROOT/gpurun_out/prof_dbg_$D -name "*kernel_stats.csv" | head -1)
  echo "DBG=$D"; grep -E "eval_|sim_kernel" "$f" | cut -d, -f1,4 | sed 's/(cmve::[^"]*//'
done
