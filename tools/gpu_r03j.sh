#!/bin/bash
# c3def (the reference's default architecture): GPU tests, then the bench line at a few step factors
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r03j; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for f in ${FACTORS:-0.02 0.005 0.002}; do
  timeout -k 10 300 python bench.py --config c3def --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --step-factor $f --accept-trajectories ${TRAJ:-3} > $OUT/c3def_$f.json 2> $OUT/c3def_$f.err || { tail $OUT/c3def_$f.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c3def_$f.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c3def f=$f', round(d['value'],3), round(d['ms_per_step'],1), 'k', round(r['kernel_ms'],1), 'acc', d['accept_rate'], d.get('accept_rate_trajectories'))"
done
