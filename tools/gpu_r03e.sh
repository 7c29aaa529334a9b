#!/bin/bash
# round 3: bench.py's own 2-rank launch on one GPU (gloo), the post-line network
# check through the library communicator, the network sampler line (multi-trajectory
# acceptance) and a kernel trace of the network sampler (forward-only vs gradient launch)
set -o pipefail
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out/r03e
mkdir -p $OUT
cd $R
BANN_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/gloo2.json 2> $OUT/gloo2.err || { tail -20 $OUT/gloo2.err; exit 1; }
cat $OUT/gloo2.json; grep network_check $OUT/gloo2.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --sampler network --step-factor 0.11 > $OUT/net.json 2> $OUT/net.err || { tail $OUT/net.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/net.json').read().strip().splitlines()[-1]); print('net', round(d['value'],1), d['accept_rate'], d.get('accept_rate_trajectories'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/nettrace -o run -- \
  python3 $R/bench.py --no-cpu-baseline --sampler network --steps 5 --warmup 2 --profile-iters 2 --step-factor 0.11 --accept-trajectories 0 > $OUT/nettrace.json 2> $OUT/nettrace.err || { echo "trace failed"; tail $OUT/nettrace.err; exit 1; }
