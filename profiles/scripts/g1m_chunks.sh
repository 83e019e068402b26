#!/bin/bash
# gallery_shard / gallery_1m with the fix-up overlapped behind the next chunk's GEMM (--chunks)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R" && mkdir -p gpurun_out/g1m_chunks || exit 1
O=gpurun_out/g1m_chunks
A="--steps 2 --warmup 1 --evals-per-step 8 --no-extras --no-cpu-baseline --no-replay --no-c3-sharded --no-c5"
for c in 1 4 8 2; do
  timeout -k 10 300 python bench.py $A --chunks $c > $O/b_c$c.json 2> $O/b_c$c.err || { echo "c$c failed"; tail -5 $O/b_c$c.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/b_c$c.json').read().strip().splitlines()[-1])
g=d['gallery_shard']; m=d['gallery_1m']
print('chunks $c', 'shard v %.4g rank ms %.3f' % (g['value'], g['rank_count']['ms']), '| 1m v %.4g rank ms %.2f mism %s' % (m['value'], m['rank_count']['ms'], m.get('sampled_rank_mismatches_vs_fp64')), 'frac', g['roofline']['frac'], m['roofline']['frac'])
"
done
