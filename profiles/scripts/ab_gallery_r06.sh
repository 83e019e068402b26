#!/bin/bash
# round 6: A/B of library variants on the gallery_shard leg (16,384 x 131,072 x 1024, G256), alternating, two passes:
#   AB_LIBS="name|lib ..." (relative to the repo; the product library is always run first as "base")
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/abg || exit 1
A="--steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-replay"
for r in 1 2; do
  for v in "base|cross-modal-video-engine_amd/cmve/libcmve.so" $AB_LIBS; do
    n=${v%%|*}; l=${v#*|}
    CMVE_LIB=$R/$l timeout -k 10 300 python bench.py $A > gpurun_out/abg/${n}_$r.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/abg/${n}_$r.log; exit 1; }
    python3 - "$n" "$r" <<'PY'
import json, sys
n, r = sys.argv[1], sys.argv[2]
d = json.loads(open(f"gpurun_out/abg/{n}_{r}.log").read().strip().splitlines()[-1])
g = d["gallery_shard"]
print(f"{n}: headline {d['value']:.4g} gallery {g['value']:.4g} ms/step {g['ms_per_step']:.3f} frac {g.get('roofline', {}).get('frac')}")
PY
  done
done
