#!/bin/bash
# N>1 rehearsal on a 1-GPU box: ranks share the GPU over gloo (bench.py --rehearse-gloo): every collective of the
# sharded path (Q all-gather, MAX / SUM all-reduces with the v2t R@K sums and the overflow flag, top-k merge)
# runs on device tensors; RCCL itself is left to the driver's node run.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out || exit 1
for n in ${REHEARSE_N:-2 4}; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 2 --rehearse-gloo --topk-leg \
    > gpurun_out/rehearse_$n.log 2>&1 || { echo "N=$n failed"; tail -20 gpurun_out/rehearse_$n.log; exit 1; }
  echo "N=$n: $(grep '^{' gpurun_out/rehearse_$n.log | tail -1 | cut -c1-300)"
done
