#!/bin/bash
# round-4 measurement pass on one MI355X (each GPU step under its own time limit, chained):
#   GPU tests, smoke(), the driver's bench line, its round profile (trace + PMC fetch / write),
#   the network-joint line and its profile, the N = 8 shard (fused update on / off),
#   C2, C5, c3def lines, the 2-rank gloo rehearsal carrying network_check
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04}; mkdir -p $OUT
P=${PTAG:-r04a}
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['value'],2), 'ms', round(d['ms_per_step'],4), 'k', round(r['kernel_ms'],4), 'frac', round(r['frac'],4), 'acc', d['accept_rate'], (d.get('accept_rate_trajectories') or {}).get('rate'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'nc', json.dumps(d.get('network_check')))"; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/c3.json 2> $OUT/c3.err || { tail $OUT/c3.err; exit 1; }
j $OUT/c3.json
bash tools/profile_round.sh $P --steps 20 --warmup 5 > $OUT/profile.log 2>&1 || { tail $OUT/profile.log; exit 1; }
grep -h "Timed trajectory" profiles/${P}_summary.md | cut -c1-400
timeout -k 10 300 python bench.py --sampler network --steps 20 --warmup 2 --no-cpu-baseline > $OUT/net.json 2> $OUT/net.err || { tail $OUT/net.err; exit 1; }
j $OUT/net.json
bash tools/profile_round.sh ${P}_net --sampler network --steps 20 --warmup 2 > $OUT/profile_net.log 2>&1 || { tail $OUT/profile_net.log; exit 1; }
for f in 1 0; do
  BANN_FUSE_UPDATE=$f timeout -k 10 300 python bench.py --emulate-shard 8 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/shard8_fuse$f.json 2> $OUT/shard8_fuse$f.err || { tail $OUT/shard8_fuse$f.err; exit 1; }
  j $OUT/shard8_fuse$f.json
done
for cfg in c2 c5 c3def; do
  timeout -k 10 400 python bench.py --config $cfg --steps 20 --warmup 2 --no-cpu-baseline > $OUT/$cfg.json 2> $OUT/$cfg.err || { tail $OUT/$cfg.err; exit 1; }
  j $OUT/$cfg.json
done
BANN_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/gloo2.json 2> $OUT/gloo2.err || { tail -20 $OUT/gloo2.err; exit 1; }
j $OUT/gloo2.json
