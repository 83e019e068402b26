#!/bin/bash
# round 6: A/B of (library, bench-argument) variants of the headline on one box, alternating, two passes:
#   AB_MIX="name|lib|args;name2|lib2|args2" (lib relative to the repo, empty = the product library)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/abm || exit 1
A="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-replay"
IFS=';' read -ra V <<< "base||;${AB_MIX}"
for r in 1 2; do
  for v in "${V[@]}"; do
    [ -z "$v" ] && continue
    n=${v%%|*}; rest=${v#*|}; l=${rest%%|*}; f=${rest#*|}
    L=${l:+$R/$l}; L=${L:-$R/cross-modal-video-engine_amd/cmve/libcmve.so}
    CMVE_LIB=$L timeout -k 10 150 python bench.py $A $f > gpurun_out/abm/${n}_$r.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/abm/${n}_$r.log; exit 1; }
    python3 - "$n" "$r" <<'PY'
import json, sys
n, r = sys.argv[1], sys.argv[2]
d = json.loads(open(f"gpurun_out/abm/{n}_{r}.log").read().strip().splitlines()[-1])
k = d.get("kernel_ms_isolated_batch") or {}
ki = d.get("kernel_ms_inflight") or {}
print(f"{n}: {d['value']:.4g} parity {d['recall']['parity_exact']} b2b {d['single_eval_back_to_back_ms']:.4f} "
      f"iso " + " ".join(f"{a}={b * 1e3:.1f}" for a, b in k.items()) + " | inflight " +
      " ".join(f"{a}={b * 1e3:.1f}" for a, b in ki.items()))
PY
  done
done
