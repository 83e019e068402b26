#!/bin/bash
# C4 fix-up: where its waves wait (SQ counters, one pass)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/c4_fixup_sq || exit 1
O=$R/gpurun_out/c4_fixup_sq
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU --kernel-trace --output-format csv -d /tmp/sqz -o run -- python3 "$R/tools/fusion_bench.py" --loop-q 0 --sample 16 > "$O/sq.log" 2>&1 || { tail -5 "$O/sq.log"; exit 1; }
python3 - /tmp/sqz <<'PY'
import collections, csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:40]
    if "fixup" in k or "sim_kernel<2" in k:
        d[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
for (k, di), v in list(d.items())[-4:]:
    wc = max(1.0, v["SQ_WAVE_CYCLES"])
    print(k, di, {c: "%.3g" % x for c, x in v.items()}, "wait_any/wave_cycles %.2f wait_inst/wave_cycles %.2f valu/wave_cycles %.3f lds %.3f vmem %.3f" % (v["SQ_WAIT_ANY"] / wc, v["SQ_WAIT_INST_ANY"] / wc, v["SQ_ACTIVE_INST_VALU"] / wc, v["SQ_ACTIVE_INST_LDS"] / wc, v["SQ_ACTIVE_INST_VMEM"] / wc))
PY
