for r in 1 2 3; do for n in 3 4; do
timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-shard-leg --no-extras --no-cpu-baseline --inflight $n --default-stream-session > gpurun_out/sd_${n}_$r.log 2>&1 || exit 1
done; done
