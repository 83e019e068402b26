# kernel study: tile-order group width (CMVE_SIM_GN) of the rank GEMM
mkdir -p gpurun_out/gn
for gn in ${GNS:-4 8 16 2}; do
  CMVE_SIM_GN=$gn MODES=F16 REPS=20 timeout -k 10 120 python tools/kbench.py > gpurun_out/gn/gn_$gn.log 2>&1 || exit 1
done
