#!/bin/bash
# bench.py's distributed path rehearsed on one GPU: `bench.py --gpus 2` starts its
# own 2 ranks (gloo callback communicator), branch and network samplers
set -o pipefail
mkdir -p gpurun_out/dist
for smp in branch network; do
  BANN_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 2 --no-cpu-baseline \
    --sampler $smp --config ${CFG:-c3} > gpurun_out/dist/bench2_$smp.json 2> gpurun_out/dist/bench2_$smp.err || { tail -20 gpurun_out/dist/bench2_$smp.err; exit 1; }
  cat gpurun_out/dist/bench2_$smp.json
done
