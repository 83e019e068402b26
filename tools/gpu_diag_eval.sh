#!/bin/bash
# K14 rank-GEMM study: rocprof kernel times of the evaluation with the diagnostic sim builds (results garbage)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
for L in FULL NOEPI NOLOAD NOFLUSH; do
  rm -rf $R/gpurun_out/diag_$L
  if [ $L = FULL ]; then LIB=$R/cross-modal-video-engine_amd/cmve/libcmve.so; else LIB=$R/diagso/libcmve_$L.so; fi
  CMVE_LIB=$LIB timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/diag_$L -o run -- python3 $R/tools/eval_bench.py --reps 100 > $R/gpurun_out/diag_$L.log 2>&1
  f=$(find $R/gpurun_out/diag_$L -name "*kernel_stats.csv" | head -1)
  echo "== $L"; grep -E "eval_|sim_kernel" "$f" | cut -d, -f1,4 | sed 's/(cmve::[^"]*//'
done
