#!/bin/bash
# round 5 (same recipe as gpu_r04b.sh): the eval parity tests, the headline at 3 / 1 streams, and a one-stream trace + FETCH /
# WRITE passes of the timed loop's batch launches (no single-set replay) -> profiles/<TAG>_1ka_*
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
TAG=${1:-r05a}
cd "$R" && mkdir -p gpurun_out/$TAG || exit 1
O=gpurun_out/$TAG
HB="--no-shard-leg --no-extras --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_retrieval.py} -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py $HB > $O/bench3.log 2>&1 || { echo "bench3 failed"; tail -20 $O/bench3.log; exit 1; }
timeout -k 10 300 python bench.py $HB --inflight 1 --no-replay > $O/bench1.log 2>&1 || { echo "bench1 failed"; tail -20 $O/bench1.log; exit 1; }
python - <<PY
import json
for f in ("bench3", "bench1"):
    d = json.loads(open("$O/%s.log" % f).read().strip().splitlines()[-1])
    print(f, "%.4g" % d["value"], "ms/step %.4f" % d["ms_per_step"], "parity", d["recall"]["parity_exact"], "undecided", d["undecided_pairs"],
          "iso gemm %.4f" % d["roofline"]["kernel_ms_live_events"], d["roofline"]["other_kernels_live_ms"], "inflight", d["kernel_ms_inflight"],
          "single %.4f b2b %.4f" % (d["single_eval_ms"], d["single_eval_back_to_back_ms"]), "replay %.4g" % d["single_set_replay"]["value"])
PY
[ -n "$NOPROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
A="$HB --inflight 1 --no-replay --steps 20 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/bench.py" $A > "$R/$O/trace.log" 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/$O/fetch" -o run -- python3 "$R/bench.py" $A > "$R/$O/fetch.log" 2>&1 || { echo "fetch failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$R/$O/write" -o run -- python3 "$R/bench.py" $A > "$R/$O/write.log" 2>&1 || { echo "write failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$R/$O/sq" -o run -- python3 "$R/bench.py" $A > "$R/$O/sq.log" 2>&1 || echo "sq pass failed (continuing)"
python3 "$R/tools/traffic_1ka.py" "$R/$O" $TAG > "$R/$O/traffic.log" 2>&1
tail -c 2500 "$R/$O/traffic.log"
