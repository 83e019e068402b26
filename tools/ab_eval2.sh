# A/B of libcmve builds on the 1k-A evaluation (kernel studies): eval_pipe + stamps per variant, two rounds
mkdir -p gpurun_out/abe2 && L=$PWD/cross-modal-video-engine_amd/cmve/ab
for r in 1 2; do for v in ${VARIANTS:-base}; do
  CMVE_LIB=$L/$v.so timeout -k 10 120 python tools/eval_pipe.py --steps 1000 > gpurun_out/abe2/pipe_${v}_$r.log 2>&1 || exit 1
  [ $r = 1 ] && { CMVE_LIB=$L/$v.so timeout -k 10 120 python tools/eval_stamps.py > gpurun_out/abe2/stamps_$v.log 2>&1 || exit 1; }
done; done
for f in gpurun_out/abe2/pipe_*.log; do echo "$f $(tail -1 $f)"; done
