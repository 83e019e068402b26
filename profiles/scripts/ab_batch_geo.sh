#!/bin/bash
# K14 batches: the batch rank GEMM's geometries (CMVE_BATCH_GEO = 64: 64 x 64, default: 128 x 64, 128128: the
# 8-wave 128 x 128), alternating; the batch tests first under each
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
GEOS=${GEOS:-"64 128 128128"}
for g in $GEOS; do
  CMVE_BATCH_GEO=$g timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_retrieval.py -k "batch" > gpurun_out/abg_test_$g.log 2>&1 || { tail -30 gpurun_out/abg_test_$g.log; exit 1; }
  echo "tests geo $g: $(tail -1 gpurun_out/abg_test_$g.log)"
done
ARGS="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-c3-sharded --no-c5 ${BATCH_ARGS:---batch 10 --inflight 2}"
for r in 1 2; do
  for g in $GEOS; do
    CMVE_BATCH_GEO=$g timeout -k 10 120 python bench.py $ARGS > gpurun_out/abgeo_${g}_$r.log 2>&1 || exit 1
    echo "$g $r: $(grep -o '"value": [0-9.e+]*' gpurun_out/abgeo_${g}_$r.log | head -1) $(grep -o '"single_set_replay": {"value": [0-9.e+]*' gpurun_out/abgeo_${g}_$r.log) $(grep -o '"parity_exact": [a-z]*' gpurun_out/abgeo_${g}_$r.log)"
  done
done
