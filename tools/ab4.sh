# A/B/C/D of libcmve builds on one box (kernel studies): interleaved kbench runs, rank pass only
mkdir -p gpurun_out/ab4 && L=$PWD/cross-modal-video-engine_amd/cmve/ab
for r in 1 2 3; do
  for v in ${VARIANTS:-base head v1 v2}; do
    KB_NOFIX=${AB_NOFIX-1} CMVE_LIB=$L/$v.so MODES=F16 REPS=30 timeout -k 10 120 python tools/kbench.py > gpurun_out/ab4/${v}_$r.log 2>&1 || exit 1
  done
done
for f in gpurun_out/ab4/*.log; do echo "$f $(grep -o '"rank_mfma_ms": [0-9.]*' $f) $(grep -o '"gemm_only_ms": [0-9.]*' $f)"; done
