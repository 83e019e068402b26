# A/B of libcmve builds on the K14 1k-A evaluation (kernel studies): eval_pipe + stamps per variant
mkdir -p gpurun_out/abe && L=$PWD/cross-modal-video-engine_amd/cmve/ab
for v in ${VARIANTS:-base defer ns4}; do
  CMVE_LIB=$L/$v.so timeout -k 10 120 python tools/eval_pipe.py --steps 400 > gpurun_out/abe/pipe_$v.log 2>&1 || exit 1
  CMVE_LIB=$L/$v.so timeout -k 10 120 python tools/eval_stamps.py > gpurun_out/abe/stamps_$v.log 2>&1 || exit 1
done
for v in ${VARIANTS:-base defer ns4}; do echo "$v $(tail -1 gpurun_out/abe/pipe_$v.log)"; done
