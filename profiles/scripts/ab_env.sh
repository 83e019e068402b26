#!/bin/bash
# round 4 A/B of environment / library variants of the headline on one box: AB_VARS="name|ENV=1 ENV2=0|lib ..." (lib
# optional, relative to the repo); prints the headline (3 / 1 streams) and the batch's isolated launch durations
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/ab || exit 1
A="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-replay ${AB_ARGS:-}"
for r in 1 2; do
  for v in "base||" $AB_VARS; do
    n=${v%%|*}; rest=${v#*|}; e=${rest%%|*}; l=${rest#*|}
    L=${l:+$R/$l}; L=${L:-$R/cross-modal-video-engine_amd/cmve/libcmve.so}
    env $e CMVE_LIB=$L timeout -k 10 150 python bench.py $A > gpurun_out/ab/${n}_b3.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/ab/${n}_b3.log; exit 1; }
    env $e CMVE_LIB=$L timeout -k 10 150 python bench.py $A --inflight 1 > gpurun_out/ab/${n}_b1.log 2>&1 || exit 1
    python3 - "$n" <<'PY'
import json, sys
n = sys.argv[1]
d3 = json.loads(open(f"gpurun_out/ab/{n}_b3.log").read().strip().splitlines()[-1])
d1 = json.loads(open(f"gpurun_out/ab/{n}_b1.log").read().strip().splitlines()[-1])
k = d1.get("kernel_ms_isolated_batch") or {}
print(f"{n}: 3s {d3['value']:.4g} 1s {d1['value']:.4g} parity {d3['recall']['parity_exact']} b2b {d3['single_eval_back_to_back_ms']:.4f} "
      f"iso(1s) " + " ".join(f"{a}={b * 1e3:.1f}" for a, b in k.items()) + f" | single {d1['kernel_ms_isolated']}")
PY
  done
done
