# K10 clock / busy counters for one metric at the measures_bench workload (PMC pass of its own)
mkdir -p gpurun_out/pmc_pw && cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$OLDPWD}
REPS=3 timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $R/gpurun_out/pmc_pw -o run -- python3 $R/tools/measures_bench.py > $R/gpurun_out/pmc_pw/log.txt 2>&1
