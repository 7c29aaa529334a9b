#!/bin/bash
# C5 step-factor sweep at the default L = 100 (bench.py's own setup): acceptance per factor
set -o pipefail
mkdir -p gpurun_out/refresh
for f in ${FACTORS:-0.1 0.07 0.05 0.03}; do
  timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --profile-iters 1 --warmup 2 --step-factor $f ${ARGS} > gpurun_out/refresh/c5_$f.json 2> gpurun_out/refresh/c5_$f.err || { tail -3 gpurun_out/refresh/c5_$f.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['accept_rate'], d['value'])" gpurun_out/refresh/c5_$f.json $f
done
