#!/bin/bash
# per-rank shard shapes of the N-GPU bench on one GPU: gradient launch time at
# 1000/N branches, then a 2-rank rehearsal of bench.py's distributed path (gloo,
# both ranks on GPU 0)
set -o pipefail
mkdir -p gpurun_out/shard
for nb in 125 250 500; do
  timeout -k 10 90 python tools/kbench.py --branches $nb --iters 30 --tag b$nb || exit 1
done
BANN_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 2 --no-cpu-baseline \
  > gpurun_out/shard/bench2.json 2> gpurun_out/shard/bench2.err || { tail -20 gpurun_out/shard/bench2.err; exit 1; }
cat gpurun_out/shard/bench2.json
