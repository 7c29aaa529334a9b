#!/bin/bash
# round-4 pass g: the remaining lines on the final tree -- N = 8 shard, C2 (+ its round
# profile), C5 (+ network check), c3def, the gloo 2-rank rehearsal, the sequential driver
set -o pipefail
R=$(pwd); T=${TAG:-r4g}; OUT=$R/gpurun_out/$T; mkdir -p $OUT; P=${PTAG:-r04b}
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['value'],2), 'ms', round(d['ms_per_step'],4), 'k', round(r['kernel_ms'],4), 'frac', round(r['frac'],4), 'acc', d['accept_rate'], (d.get('accept_rate_trajectories') or {}).get('rate'), 'nc', json.dumps(d.get('network_check')))"; }
timeout -k 10 300 python bench.py --emulate-shard 8 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/shard8.json 2> $OUT/shard8.err || { tail $OUT/shard8.err; exit 1; }
j $OUT/shard8.json
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err || { tail $OUT/c2.err; exit 1; }
j $OUT/c2.json
bash tools/profile_round.sh ${P}_c2 --config c2 --steps 20 --warmup 5 --no-network-check > $OUT/profile_c2.log 2>&1 || { tail $OUT/profile_c2.log; exit 1; }
timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err || { tail $OUT/c5.err; exit 1; }
j $OUT/c5.json
timeout -k 10 400 python bench.py --config c3def --steps 20 --warmup 2 --no-cpu-baseline --no-network-check > $OUT/c3def.json 2> $OUT/c3def.err || { tail $OUT/c3def.err; exit 1; }
j $OUT/c3def.json
BANN_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/gloo2.json 2> $OUT/gloo2.err || { tail -20 $OUT/gloo2.err; exit 1; }
j $OUT/gloo2.json
timeout -k 10 300 python bench.py --sampler sequential --steps 20 --warmup 0 --no-cpu-baseline > $OUT/seq.json 2> $OUT/seq.err || { tail $OUT/seq.err; exit 1; }
j $OUT/seq.json
