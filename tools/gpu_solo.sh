#!/bin/bash
# full GPU suite + the sequential driver bench lines (solo-mode plans)
set -o pipefail
LIMIT=600 bash tools/gpu_tests.sh | tail -3 || exit 1
mkdir -p gpurun_out/seq
for c in c3 c2; do
  timeout -k 10 300 python bench.py --config $c --sampler sequential --no-cpu-baseline > gpurun_out/seq/${c}seq.json 2> gpurun_out/seq/${c}seq.err || { tail -5 gpurun_out/seq/${c}seq.err; exit 1; }
  python3 -c "import json;b=json.load(open('gpurun_out/seq/${c}seq.json'));print('$c sequential',b['value'],b['ms_per_step'],b['accept_rate'])"
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/seq/c3.json 2> gpurun_out/seq/c3.err || exit 1
python3 -c "import json;b=json.load(open('gpurun_out/seq/c3.json'));print('c3 packed',b['value'],b['ms_per_step'],b['accept_rate'])"
