#!/bin/bash
# round 4, first box: counter calibration, the headline with the streams on distinct input groups (3 and 1
# in flight), and a one-stream trace + FETCH / WRITE passes of the batch launches
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/r04a || exit 1
O=gpurun_out/r04a
HB="--no-shard-leg --no-extras --no-cpu-baseline"
timeout -k 10 300 bash profiles/scripts/calib.sh > $O/calib.log 2>&1 || { echo "calib failed"; tail -20 $O/calib.log; exit 1; }
cat $O/calib.log
timeout -k 10 300 python bench.py $HB > $O/bench3.log 2>&1 || { echo "bench3 failed"; tail -20 $O/bench3.log; exit 1; }
timeout -k 10 300 python bench.py $HB --inflight 1 > $O/bench1.log 2>&1 || { echo "bench1 failed"; tail -20 $O/bench1.log; exit 1; }
python - <<'PY'
import json
for f in ("bench3", "bench1"):
    d = json.loads(open(f"gpurun_out/r04a/{f}.log").read().strip().splitlines()[-1])
    print(f, "%.4g" % d["value"], d["ms_per_step"], "iso", d["roofline"]["kernel_ms_live_events"], d["roofline"]["other_kernels_live_ms"], "inflight", d["kernel_ms_inflight"])
PY
cd /tmp && export TMPDIR=/tmp
A="$HB --inflight 1 --steps 20 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace" -o run -- python3 "$R/bench.py" $A > "$R/$O/trace.log" 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/$O/fetch" -o run -- python3 "$R/bench.py" $A > "$R/$O/fetch.log" 2>&1 || { echo "fetch failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$R/$O/write" -o run -- python3 "$R/bench.py" $A > "$R/$O/write.log" 2>&1 || { echo "write failed"; exit 1; }
python3 "$R/tools/traffic_1ka.py" "$R/$O" r04a > "$R/$O/traffic.log" 2>&1
tail -c 2500 "$R/$O/traffic.log"
