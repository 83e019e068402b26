# A/B of two builds of libcmve on one box (kernel studies): ABAB kbench runs, rank pass only
mkdir -p gpurun_out/ab && L=$PWD/cross-modal-video-engine_amd
A=${A:-$L/build/libcmve_base.so}; B=${B:-$L/cmve/libcmve.so}
for r in 1 2 3; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    KB_NOFIX=${AB_NOFIX-1} CMVE_LIB=$lib MODES=F16 REPS=30 timeout -k 10 120 python tools/kbench.py > gpurun_out/ab/${v}_$r.log 2>&1 || exit 1
  done
done
for f in gpurun_out/ab/*.log; do echo "$f $(grep -o '"rank_mfma_ms": [0-9.]*' $f) $(grep -o '"gemm_only_ms": [0-9.]*' $f) $(grep -o '"fixup_ms": [0-9.]*' $f)"; done
