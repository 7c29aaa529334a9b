#!/bin/bash
# round-4 pass d: the network tests, the C3 network line with the network error read by the
# gradient kernel (default) vs per-branch targets (BANN_NET_ERR=0), the C5 network sampler at
# small factors
set -o pipefail
R=$(pwd); T=${TAG:-r4d}; OUT=$R/gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_network_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log | cut -c1-400; exit 1; }
tail -1 $OUT/tests.log
TAG=$T/net VARIANTS="- BANN_NET_ERR=0 BANN_FWD_FI=0 BANN_FWD_FI=0,BANN_NET_ERR=0" BARGS="--sampler network --steps 20 --warmup 2" bash tools/gpu_c3ab.sh || exit 1
for f in ${C5F:-0.0005 0.001}; do
  timeout -k 10 300 python bench.py --config c5 --sampler network --step-factor $f --steps 20 --warmup 0 --accept-trajectories 1 --no-cpu-baseline > $OUT/c5net_$f.json 2> $OUT/c5net_$f.err || { tail $OUT/c5net_$f.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/c5net_$f.json').read().strip().splitlines()[-1]); print('c5net $f', round(d['value'],3), d['accept_rate'], d.get('accept_rate_trajectories'))"
done
