#!/bin/bash
# round-6 pass on the current tree, in two parts (each within one gpurun call):
#   PART=a: GPU tests, smoke, the driver's C3 line and its round profile, the network line and its profile
#   PART=b: the N = 8 shard, the gloo 2-rank rehearsal, C2, C5, c3def, the sequential driver
set -o pipefail
R=$(pwd); T=${TAG:-r06}; OUT=$R/gpurun_out/$T; mkdir -p $OUT; P=${PTAG:-r06}
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; nc=d.get('network_check') or {}; nt=d.get('network_timing') or {}; print('$1', round(d['value'],2), 'ms', round(d['ms_per_step'],4), 'k', round(r['kernel_ms'],4), 'frac', round(r['frac'],4), 'acc', d['accept_rate'], (d.get('accept_rate_trajectories') or {}).get('rate'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'nc', nc.get('status'), nc.get('steps_per_s'), 'fwd', nt.get('forward_ms') or nc.get('forward_ms'))"; }
if [ "${PART:-a}" = a ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/c3.json 2> $OUT/c3.err || { tail $OUT/c3.err; exit 1; }
j $OUT/c3.json
bash tools/profile_round.sh $P --steps 20 --warmup 5 > $OUT/profile.log 2>&1 || { tail $OUT/profile.log; exit 1; }
timeout -k 10 300 python bench.py --sampler network --steps 20 --warmup 2 --no-cpu-baseline --accept-trajectories 9 > $OUT/net.json 2> $OUT/net.err || { tail $OUT/net.err; exit 1; }
j $OUT/net.json
bash tools/profile_round.sh ${P}_net --sampler network --steps 20 --warmup 2 > $OUT/profile_net.log 2>&1 || { tail $OUT/profile_net.log; exit 1; }
else
timeout -k 10 300 python bench.py --emulate-shard 8 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/shard8.json 2> $OUT/shard8.err || { tail $OUT/shard8.err; exit 1; }
j $OUT/shard8.json
BANN_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/gloo2.json 2> $OUT/gloo2.err || { tail -20 $OUT/gloo2.err; exit 1; }
j $OUT/gloo2.json
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err || { tail $OUT/c2.err; exit 1; }
j $OUT/c2.json
timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err || { tail $OUT/c5.err; exit 1; }
j $OUT/c5.json
timeout -k 10 400 python bench.py --config c3def --steps 20 --warmup 2 --no-cpu-baseline --no-network-check > $OUT/c3def.json 2> $OUT/c3def.err || { tail $OUT/c3def.err; exit 1; }
j $OUT/c3def.json
timeout -k 10 400 python bench.py --sampler sequential --steps 20 --warmup 2 --no-cpu-baseline --no-network-check > $OUT/seq.json 2> $OUT/seq.err || { tail $OUT/seq.err; exit 1; }
j $OUT/seq.json
fi
