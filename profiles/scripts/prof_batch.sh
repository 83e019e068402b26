#!/bin/bash
# K14 batches: kernel trace (one stream: isolated kernel durations) + an L2 counter pass of the same loop
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R" && mkdir -p gpurun_out || exit 1
T=${TAG:-b}
ARGS="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-c3-sharded --no-c5 ${BATCH_ARGS:---batch 10 --inflight 1}"
rm -rf gpurun_out/prof_$T gpurun_out/pmc_$T
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- python3 bench.py $ARGS > gpurun_out/prof_$T.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/pmc_$T -o run -- python3 bench.py $ARGS --steps 5 --warmup 2 > gpurun_out/pmc_$T.log 2>&1 || exit 1
python3 - "$T" <<'PY'
import csv, collections, statistics, sys
t = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/prof_{t}/run_kernel_stats.csv")):
    if "batch" in r["Name"] or "true>" in r["Name"]:
        print(f"{r['Name'][:64]:66s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.2f} us min {float(r['MinNs'])/1e3:8.2f}")
d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f"gpurun_out/pmc_{t}/run_counter_collection.csv")):
    if "batch" in r["Kernel_Name"] or "true>" in r["Kernel_Name"]:
        d[r["Kernel_Name"][:64]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in d.items():
    m = {c: statistics.median(x) for c, x in v.items()}
    print(f"{k:66s} " + " ".join(f"{c} {x:.0f}" for c, x in m.items()) + f" hit {m['TCC_HIT_sum']/max(1,m['TCC_REQ_sum']):.2f}")
PY
