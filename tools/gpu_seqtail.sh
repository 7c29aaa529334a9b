#!/bin/bash
# sequential-driver tail (hmc_step_tail): the driver's GPU tests, then the sequential line twice
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-seqtail}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest ${SEL:-tests/test_net_driver.py tests/test_effect_sizes_gpu.py} -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --sampler sequential --steps 20 --warmup 0 --no-cpu-baseline > $OUT/seq_$r.json 2> $OUT/seq_$r.err || { tail $OUT/seq_$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/seq_$r.json').read().strip().splitlines()[-1]); print('seq', round(d['value'],3), 'ms', round(d['ms_per_step'],3), 'acc', d['accept_rate'])"
done
