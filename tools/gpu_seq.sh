#!/bin/bash
# bench lines: c3def at L = 20 (accepting step factor), the sequential Net::train driver on C3 and C2
set -o pipefail
mkdir -p gpurun_out/seq
timeout -k 10 400 python bench.py --config c3def --steps 20 --warmup 2 --profile-iters 3 > gpurun_out/seq/c3def.json 2> gpurun_out/seq/c3def.err || { tail -5 gpurun_out/seq/c3def.err; exit 1; }
cat gpurun_out/seq/c3def.json
timeout -k 10 300 python bench.py --sampler sequential --no-cpu-baseline > gpurun_out/seq/c3seq.json 2> gpurun_out/seq/c3seq.err || { tail -5 gpurun_out/seq/c3seq.err; exit 1; }
cat gpurun_out/seq/c3seq.json
timeout -k 10 300 python bench.py --config c2 --sampler sequential --no-cpu-baseline > gpurun_out/seq/c2seq.json 2> gpurun_out/seq/c2seq.err || { tail -5 gpurun_out/seq/c2seq.err; exit 1; }
cat gpurun_out/seq/c2seq.json
