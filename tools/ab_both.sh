# A/B of two libcmve builds (kernel studies): kbench rank pass (gallery shape) + eval_pipe (1k-A), interleaved
L=$PWD/cross-modal-video-engine_amd/cmve/ab; mkdir -p gpurun_out/abb
for r in 1 2; do for v in ${VARIANTS:-base direct}; do
  KB_NOFIX=${AB_NOFIX-1} CMVE_LIB=$L/$v.so MODES=F16 REPS=30 timeout -k 10 120 python tools/kbench.py > gpurun_out/abb/kb_${v}_$r.log 2>&1 || exit 1
  CMVE_LIB=$L/$v.so timeout -k 10 120 python tools/eval_pipe.py --steps 1000 > gpurun_out/abb/pipe_${v}_$r.log 2>&1 || exit 1
done; done
for f in gpurun_out/abb/kb_*.log; do echo "$f $(grep -o '"rank_mfma_ms": [0-9.]*' $f)"; done
for f in gpurun_out/abb/pipe_*.log; do echo "$f $(tail -1 $f)"; done
