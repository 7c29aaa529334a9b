#!/bin/bash
# round 3: tests (graph replay of bann_hmc_step, fold kernel), C3 line, network
# factor, sequential driver with / without graph replay
set -o pipefail
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out/r03c
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -5 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['value'],1), round(d['ms_per_step'],4), 'acc', d['accept_rate'], 'fx', round(r['kernel_ms'],4), 'b2b', round(r.get('kernel_ms_back_to_back',0),4), 'upd', round(r['update_kernel_ms'],4))"; }
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/c3.json 2> $OUT/c3.err || { tail $OUT/c3.err; exit 1; }
j $OUT/c3.json
for f in 0.12 0.15; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --sampler network --step-factor $f > $OUT/net_$f.json 2> $OUT/net_$f.err || { tail $OUT/net_$f.err; exit 1; }
  j $OUT/net_$f.json
done
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --sampler sequential > $OUT/seq.json 2> $OUT/seq.err || { tail $OUT/seq.err; exit 1; }
j $OUT/seq.json
BANN_HMC_GRAPH=1 timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --sampler sequential > $OUT/seq_nog.json 2> $OUT/seq_nog.err || { tail $OUT/seq_nog.err; exit 1; }
j $OUT/seq_nog.json
