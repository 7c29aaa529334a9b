#!/bin/bash
# gx (layered MFMA) path: c3def bench line + kernel trace (output under gpurun_out/gx)
# (L = 3: Izmailov factor 0.005 accepts every branch; 0.02 is the L = 20 choice, tools/c5_accept.py)
set -o pipefail
mkdir -p gpurun_out/gx
R=$(pwd)
timeout -k 10 300 python bench.py --config c3def --steps ${STEPS:-3} --warmup 1 --profile-iters 3 --step-factor ${FACTOR:-0.005} ${ARGS} > gpurun_out/gx/bench.json 2> gpurun_out/gx/bench.err || { tail -5 gpurun_out/gx/bench.err; exit 1; }
cat gpurun_out/gx/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/gx/trace -o gx -- \
  python3 $R/bench.py --config c3def --steps 2 --warmup 1 --profile-iters 2 --step-factor ${FACTOR:-0.005} --no-cpu-baseline > $R/gpurun_out/gx/trace_bench.json 2> $R/gpurun_out/gx/trace.err || { tail -5 $R/gpurun_out/gx/trace.err; exit 1; }
find $R/gpurun_out/gx/trace -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
