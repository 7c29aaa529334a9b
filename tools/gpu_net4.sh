#!/bin/bash
# network-sampler pass: GPU tests, the C3 network line with the fi forward on / off
# (BANN_FWD_FI), and the C5 network sampler's acceptance at two step factors
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-net4}; mkdir -p $OUT
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['value'],2), 'ms', round(d['ms_per_step'],4), 'k', round(r['kernel_ms'],4), 'acc', d['accept_rate'], (d.get('accept_rate_trajectories') or {}).get('rate'), 'nc', json.dumps(d.get('network_check')))"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in 1 0 1; do
  BANN_FWD_FI=$v timeout -k 10 300 python bench.py --sampler network --steps 20 --warmup 2 --no-cpu-baseline > $OUT/net_fi$v.json 2> $OUT/net_fi$v.err || { tail $OUT/net_fi$v.err; exit 1; }
  j $OUT/net_fi$v.json
done
for f in ${C5F:-0.002 0.005}; do
  timeout -k 10 400 python bench.py --config c5 --sampler network --step-factor $f --steps 20 --warmup 0 --accept-trajectories 2 --no-cpu-baseline > $OUT/c5net_$f.json 2> $OUT/c5net_$f.err || { tail $OUT/c5net_$f.err; exit 1; }
  j $OUT/c5net_$f.json
done
