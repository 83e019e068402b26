#!/bin/bash
# G256 rank GEMM study (16,384 x 131,072 x 1024, F16): the product kernel, the no-epilogue diagnostic build,
# and the per-block stamps build (prologue / main loop / epilogue pieces).  Diagnostic libraries are built
# in this container (make diag DIAG=NOEPI / STAMPS) and copied to diaglib/.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
KB_NOFIX=1 MODES=F16 REPS=10 timeout -k 10 150 python tools/kbench.py > gpurun_out/g256_full.log 2>&1 \
  && KB_NOFIX=1 CMVE_LIB=$R/diaglib/libcmve_NOEPI.so MODES=F16 REPS=10 timeout -k 10 150 python tools/kbench.py > gpurun_out/g256_noepi.log 2>&1 \
  && KB_STAMPS=real CMVE_LIB=$R/diaglib/libcmve_STAMPS.so MODES=F16 REPS=3 timeout -k 10 150 python tools/kbench.py > gpurun_out/g256_stamps.log 2>&1
rc=$?
for f in full noepi stamps; do echo "== $f"; grep -v probe gpurun_out/g256_$f.log | grep "^{" | head -4; done
exit $rc
