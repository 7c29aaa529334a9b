#!/bin/bash
# bench.py's distributed path rehearsed on one GPU: 2 ranks over gloo (library
# callback communicator), branch and network samplers; then the 1-GPU network line
set -o pipefail
mkdir -p gpurun_out/dist
for smp in branch network; do
  BANN_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 2 --no-cpu-baseline \
    --sampler $smp --config ${CFG:-c3} > gpurun_out/dist/bench2_$smp.json 2> gpurun_out/dist/bench2_$smp.err || { tail -20 gpurun_out/dist/bench2_$smp.err; exit 1; }
  cat gpurun_out/dist/bench2_$smp.json
done
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --sampler network --config ${CFG:-c3} \
  > gpurun_out/dist/bench1_network.json 2> gpurun_out/dist/bench1_network.err || { tail -20 gpurun_out/dist/bench1_network.err; exit 1; }
cat gpurun_out/dist/bench1_network.json
