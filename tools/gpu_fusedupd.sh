#!/bin/bash
# GPU tests, then the C3 bench with and without the update fused into the fx launch
set -o pipefail
bash tools/gpu_tests.sh || exit 1
mkdir -p gpurun_out/fu
for r in 1 2; do
  for f in 1 0; do
    BANN_FUSED_UPDATE=$f timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/fu/c3_$f.json 2> gpurun_out/fu/c3_$f.err || { tail -3 gpurun_out/fu/c3_$f.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('fused', sys.argv[2], round(d['value'],2), round(d['ms_per_step'],4), d['accept_rate'])" gpurun_out/fu/c3_$f.json $f
  done
done
