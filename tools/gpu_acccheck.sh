#!/bin/bash
# acceptance check after a bench setup change: C3 (L = 20), C5 factors, c3def
set -o pipefail
mkdir -p gpurun_out/refresh
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/refresh/c3q.json 2> gpurun_out/refresh/c3q.err || { tail -3 gpurun_out/refresh/c3q.err; exit 1; }
grep -o '"accept_rate[^,]*' gpurun_out/refresh/c3q.json
FACTORS="${C5F:-0.1 0.2}" bash tools/gpu_c5sweep.sh || exit 1
bash tools/gpu_gx.sh
