for r in 1 2; do for n in 2 3 4 6 8; do
timeout -k 10 100 python bench.py --no-shard-leg --no-extras --no-cpu-baseline --inflight $n > gpurun_out/sw_${n}_$r.log 2>&1 || exit 1
done; done
