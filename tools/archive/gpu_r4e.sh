#!/bin/bash
# round-4 pass e: the network line after the bench fix (the profile session no longer moves
# the chain): defaults (LDS forward, the kernel reads the network error) vs per-branch
# targets vs the fi forward, with -H traces; the C3 branch line with its network_check
set -o pipefail
R=$(pwd); T=${TAG:-r4e}; OUT=$R/gpurun_out/$T; mkdir -p $OUT
BANN_BENCH_TRACE=1 TAG=$T/net VARIANTS="- BANN_NET_ERR=0 BANN_FWD_FI=1" BARGS="--sampler network --steps 20 --warmup 2" bash tools/gpu_c3ab.sh || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/c3.json 2> $OUT/c3.err || { tail $OUT/c3.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/c3.json').read().strip().splitlines()[-1]); print('c3', round(d['value'],2), d['accept_rate'], json.dumps(d.get('network_check')))"
