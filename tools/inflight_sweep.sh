# 1k-A headline: evaluations in flight, three runs each at the driver's --steps 20 (kernel studies)
for r in 1 2 3; do for n in ${SWEEP_N:-2 3 4 6 8}; do
timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --inflight $n > gpurun_out/sw_${n}_$r.log 2>&1 || exit 1
done; done
