# kernel study: the product kernel and its no-load / no-MFMA diagnostic builds (tools/kbench.py)
mkdir -p gpurun_out/diag && L=$PWD/cross-modal-video-engine_amd/build
GEOS=${GEOS:-"0"}
for geo in $GEOS; do
  for lib in NOLOAD NOMFMA; do
    KB_NOFIX=1 CMVE_SIM_GEO=$geo CMVE_LIB=$L/libcmve_$lib.so MODES=F16 REPS=20 timeout -k 10 120 python tools/kbench.py > gpurun_out/diag/${lib}_${geo}.log 2>&1 || exit 1
  done
  CMVE_SIM_GEO=$geo MODES=F16 REPS=20 timeout -k 10 120 python tools/kbench.py > gpurun_out/diag/FULL_${geo}.log 2>&1 || exit 1
done
