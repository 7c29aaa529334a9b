#!/bin/bash
# C5 bench lines at the default L = 100 (the step factor 0.15 is sized for it): f32 and bf16 hidden GEMMs
set -o pipefail
mkdir -p gpurun_out/refresh
O=gpurun_out/refresh
timeout -k 10 400 python bench.py --config c5 > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
cat $O/c5.json
timeout -k 10 300 python bench.py --config c5 --hidden-bf16 --no-cpu-baseline > $O/c5bf.json 2> $O/c5bf.err || { tail -5 $O/c5bf.err; exit 1; }
cat $O/c5bf.json
