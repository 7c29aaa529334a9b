#!/bin/bash
# network sampler: group-sum forward tests, then the network line per variant (alternating)
# VARIANTS: env assignments separated by spaces, "-" = none
set -o pipefail
R=$(pwd); T=${TAG:-r06net}; OUT=$R/gpurun_out/$T; mkdir -p $OUT
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; nt=d.get('network_timing') or {}; print('$1', round(d['value'],2), 'ms', round(d['ms_per_step'],4), 'grad', round(r['kernel_ms'],4), 'fwd', nt.get('forward_ms'), 'acc', (d.get('accept_rate_trajectories') or {}).get('rate'))"; }
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_network_gpu.py -m gpu > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
fi
for i in $(seq 1 ${REPS:-2}); do
k=0
for v in ${VARIANTS:-"-"}; do
k=$((k+1))
f=$OUT/net_${k}_$i
if [ "$v" = "-" ]; then E=""; else E="$v"; fi
env $E timeout -k 10 300 python bench.py --sampler network --steps 20 --warmup 2 --no-cpu-baseline --accept-trajectories ${ACC:-2} > $f.json 2> $f.err || { tail $f.err; exit 1; }
echo -n "$v "; j $f.json
done
done
