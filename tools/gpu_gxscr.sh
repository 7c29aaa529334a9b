#!/bin/bash
# c3def gradient time vs the gx scratch budget (branches per group)
set -o pipefail
mkdir -p gpurun_out/gs
for mb in 8192 16384 32768; do
  BANN_GX_SCRATCH_MB=$mb timeout -k 10 300 python bench.py --config c3def --steps 3 --warmup 1 --profile-iters 3 --step-factor 0.005 --no-cpu-baseline > gpurun_out/gs/s$mb.json 2> gpurun_out/gs/s$mb.err || { tail -3 gpurun_out/gs/s$mb.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('scratch', sys.argv[2], round(d['value'],3), round(r['kernel_ms'],2), round(r['frac'],3), d['accept_rate'])" gpurun_out/gs/s$mb.json $mb
done
