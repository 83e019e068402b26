#!/bin/bash
# round 4 A/B on one box: the headline (3 and 1 streams) and the batch stamps for the product library and each
# study library of AB_LIBS="name:path ...", alternating twice
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out/ab || exit 1
A="--steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --no-replay ${AB_ARGS:-}"
one() {  # name lib
  local n=$1 l=$2
  CMVE_LIB=$l timeout -k 10 150 python bench.py $A > gpurun_out/ab/${n}_b3.log 2>&1 || { echo "$n bench failed"; tail -5 gpurun_out/ab/${n}_b3.log; return 1; }
  CMVE_LIB=$l timeout -k 10 150 python bench.py $A --inflight 1 > gpurun_out/ab/${n}_b1.log 2>&1 || return 1
  CMVE_LIB=$l timeout -k 10 120 python tools/batch_stamps.py > gpurun_out/ab/${n}_st.log 2>&1 || return 1
  python3 - "$n" <<'PY'
import json, sys, re
n = sys.argv[1]
d3 = json.loads(open(f"gpurun_out/ab/{n}_b3.log").read().strip().splitlines()[-1])
d1 = json.loads(open(f"gpurun_out/ab/{n}_b1.log").read().strip().splitlines()[-1])
st = open(f"gpurun_out/ab/{n}_st.log").read()
j = json.loads(st[st.index("{"):])
g = j["gemm"]
print(f"{n}: 3s {d3['value']:.4g} 1s {d1['value']:.4g} parity {d3['recall']['parity_exact']} iso {d3['roofline']['kernel_ms_live_events']:.4f} "
      f"prep {d3['roofline']['other_kernels_live_ms']['pack_gt_scores']:.4f} b2b {d3['single_eval_back_to_back_ms']:.4f} | gemm span "
      f"{g['end_last'] - g['start_first']:.1f} tile p50 {g['tile_p50']:.1f} loop {g['loop_med']:.1f} emit {g['emit_med']:.1f} "
      f"inflight {g['inflight_med']:.0f} prep {j['prep']['end_last']:.1f}")
PY
}
for r in 1 2; do
  one base "$R/cross-modal-video-engine_amd/cmve/libcmve.so" || exit 1
  for v in $AB_LIBS; do one "${v%%:*}" "$R/${v#*:}" || exit 1; done
done
