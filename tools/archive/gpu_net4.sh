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
# C3 branch sampler: the update in the gradient launch's tail (default for one-split plans) vs its own launch
for v in def 0 def 0; do
  if [ $v = def ]; then E="env -u BANN_FUSE_UPDATE"; else E="env BANN_FUSE_UPDATE=0"; fi
  $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c3_fuse$v.json 2> $OUT/c3_fuse$v.err || { tail $OUT/c3_fuse$v.err; exit 1; }
  j $OUT/c3_fuse$v.json
done
# C2: fxl with 4 chunks per wave and resident digit operands (default) vs 8 chunks per wave (BANN_FXL_CPW=8)
for v in 4 8 4; do
  BANN_FXL_CPW=$v timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline --no-network-check > $OUT/c2_cpw$v.json 2> $OUT/c2_cpw$v.err || { tail $OUT/c2_cpw$v.err; exit 1; }
  j $OUT/c2_cpw$v.json
done
