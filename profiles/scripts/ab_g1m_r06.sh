#!/bin/bash
# round 6: A/B of library variants on the gallery_1m leg (16,384 x 1,048,576 x 1024 in --g1m-chunks chunks, each
# chunk's fix-up behind the next chunk's G256 launch), alternating, two passes: AB_LIBS="name|lib ..."
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/ab1m || exit 1
A="--steps 3 --warmup 1 --evals-per-step 8 --no-extras --no-cpu-baseline --no-replay --no-c3-sharded --no-c5 --no-gallery-shard"
for r in 1 2; do
  for v in "base|cross-modal-video-engine_amd/cmve/libcmve.so" $AB_LIBS; do
    n=${v%%|*}; l=${v#*|}
    CMVE_LIB=$R/$l timeout -k 10 300 python bench.py $A > gpurun_out/ab1m/${n}_$r.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab1m/${n}_$r.log; exit 1; }
    python3 - "$n" "$r" <<'PY'
import json, sys
n, r = sys.argv[1], sys.argv[2]
d = json.loads(open(f"gpurun_out/ab1m/{n}_{r}.log").read().strip().splitlines()[-1])
m = d["gallery_1m"]
print(f"{n}: gallery_1m {m['value']:.4g} ms/step {m['ms_per_step']:.2f} mismatches {m.get('sampled_rank_mismatches_vs_fp64')}")
PY
  done
done
