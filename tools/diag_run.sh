mkdir -p gpurun_out/diag && L=$PWD/cross-modal-video-engine_amd/build
for lib in NOLOAD NOMFMA; do
  for geo in 2562 128; do
    KB_NOFIX=1 CMVE_SIM_GEO=$geo CMVE_LIB=$L/libcmve_$lib.so MODES=F16 REPS=20 timeout -k 10 120 python tools/kbench.py > gpurun_out/diag/${lib}_${geo}.log 2>&1 || exit 1
  done
done
CMVE_SIM_GEO=2562 MODES=F16 REPS=20 timeout -k 10 120 python tools/kbench.py > gpurun_out/diag/FULL_2562.log 2>&1
