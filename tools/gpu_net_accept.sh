#!/bin/bash
# network-joint sampler acceptance vs step factor (bench.py --sampler network, one line per factor):
#   CFG=c3 FACTORS="0.5 1.0" RULE=common_mode TRAJ=9 bash tools/gpu_net_accept.sh
set -o pipefail
OUT=gpurun_out/${TAG:-netacc}; mkdir -p $OUT
for f in ${FACTORS:-1.0}; do
  timeout -k 10 ${TMO:-300} python bench.py --config ${CFG:-c3} --sampler network --steps ${L:-20} --warmup ${W:-2} \
    --no-cpu-baseline --accept-trajectories ${TRAJ:-9} --step-factor $f --network-step-rule ${RULE:-common_mode} \
    > $OUT/${CFG:-c3}_$f.json 2> $OUT/${CFG:-c3}_$f.err || { tail -3 $OUT/${CFG:-c3}_$f.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/${CFG:-c3}_$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value'],2), d['accept_rate_trajectories'], d.get('network_step_rule'))"
done
