#!/bin/bash
# study: fp64 butterfly on the VALU (DPP / permlane swaps) vs ds_bpermute, C4 ranking + gallery shard + 1M fix-up
# (build the study library first: the Makefile objects with -DCMVE_STUDY_DPP=1 linked into scratch/libcmve_dpp.so)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/fixup_dpp || exit 1
O=gpurun_out/fixup_dpp
CMVE_LIB=$R/scratch/libcmve_dpp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fixup_tiled.py -x -q --timeout 150 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -ne 0 ] && exit $rc
for cfg in "base|" "dpp|$R/scratch/libcmve_dpp.so" "base2|" "dpp2|$R/scratch/libcmve_dpp.so"; do
  n=${cfg%%|*}; lib=${cfg#*|}
  if [ -n "$lib" ]; then export CMVE_LIB=$lib; else unset CMVE_LIB; fi
  timeout -k 10 240 python tools/fusion_bench.py --loop-q 0 --sample 64 > $O/c4_$n.json 2> $O/c4_$n.err || { echo "c4 $n failed"; tail -5 $O/c4_$n.err; exit 1; }
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --evals-per-step 8 --no-extras --no-cpu-baseline --no-replay --no-c3-sharded --no-c5 --g1m-chunks 1 > $O/b_$n.json 2> $O/b_$n.err || { echo "b $n failed"; tail -5 $O/b_$n.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c4_$n.json').read().strip().splitlines()[-1]); r=d['ranking']
b=json.loads(open('$O/b_$n.json').read().strip().splitlines()[-1]); g=b['gallery_shard']; m=b['gallery_1m']
print('$n', 'c4 rank ms %.2f mism %d' % (r['ms'], r['fp64_sample']['mismatches']), '| shard fix ms %.3f' % g['rank_count']['fixup_ms'], '| 1m fix ms %.2f mism %s' % (m['rank_count']['fixup_ms'], m['sampled_rank_mismatches_vs_fp64']), 'headline parity', b['recall']['parity_exact'])
"
done
