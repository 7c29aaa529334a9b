#!/bin/bash
# round-4 pass c (one box, every step under its own limit, chained): GPU tests; the C3
# network line with the fi forward on / off; the C5 network sampler at two factors; C2 with
# 4 vs 8 chunks per fxl wave; the fused-update A/Bs (sequential driver, C3, N = 8 shard)
set -o pipefail
R=$(pwd); T=${TAG:-r4c}; OUT=$R/gpurun_out/$T; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
TAG=$T/net VARIANTS="- BANN_FWD_FI=0" BARGS="--sampler network --steps 20 --warmup 2" bash tools/gpu_c3ab.sh || exit 1
TAG=$T/seq VARIANTS="- BANN_FUSE_UPDATE=0,BANN_SOLO_TPW=1" BARGS="--sampler sequential --steps 20 --warmup 0" bash tools/gpu_c3ab.sh || exit 1
TAG=$T/c3 VARIANTS="- BANN_FUSE_UPDATE=1" bash tools/gpu_c3ab.sh || exit 1
TAG=$T/shard VARIANTS="- BANN_FUSE_UPDATE=1" BARGS="--emulate-shard 8 --steps 20 --warmup 5" bash tools/gpu_c3ab.sh || exit 1
TAG=$T/c2 VARIANTS="- BANN_FXL_CPW=8" BARGS="--config c2 --steps 20 --warmup 5" bash tools/gpu_c3ab.sh || exit 1
for f in ${C5F:-0.002 0.005}; do
  timeout -k 10 300 python bench.py --config c5 --sampler network --step-factor $f --steps 20 --warmup 0 --accept-trajectories 1 --no-cpu-baseline > $OUT/c5net_$f.json 2> $OUT/c5net_$f.err || { tail $OUT/c5net_$f.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/c5net_$f.json').read().strip().splitlines()[-1]); print('c5net $f', round(d['value'],3), d['accept_rate'], d.get('accept_rate_trajectories'))"
done
