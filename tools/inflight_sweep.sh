# 1k-A headline: evaluations in flight x (graph replay | direct enqueue), two runs each (kernel studies)
for r in 1 2; do for n in ${SWEEP_N:-2 3 4 6}; do for gflag in "" "--graphs"; do
timeout -k 10 100 python bench.py --no-shard-leg --no-extras --no-cpu-baseline --inflight $n $gflag > gpurun_out/sw_${n}${gflag}_$r.log 2>&1 || exit 1
done; done; done
