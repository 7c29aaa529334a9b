#!/bin/bash
# C5 (4k branches x 125 SNPs, n = 100k, W = S = 32) on one GPU: fp32 and bf16
# hidden-GEMM bench lines + a kernel-trace profile of the fp32 run.
set -o pipefail
mkdir -p gpurun_out/c5
timeout -k 10 300 python bench.py --config c5 --steps ${STEPS:-50} --warmup 5 --cpu-sample-branches 16 --cpu-sample-steps 4 \
  > gpurun_out/c5/f32.json 2> gpurun_out/c5/f32.err || { tail gpurun_out/c5/f32.err; exit 1; }
cat gpurun_out/c5/f32.json
timeout -k 10 300 python bench.py --config c5 --steps ${STEPS:-50} --warmup 5 --hidden-bf16 --no-cpu-baseline \
  > gpurun_out/c5/bf16.json 2> gpurun_out/c5/bf16.err || { tail gpurun_out/c5/bf16.err; exit 1; }
cat gpurun_out/c5/bf16.json
[ -n "$NOPROF" ] && exit 0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c5/trace -o c5 -- \
  python3 $R/bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline > $R/gpurun_out/c5/trace.json 2> $R/gpurun_out/c5/trace.err \
  || { tail $R/gpurun_out/c5/trace.err; exit 1; }
echo profiled
