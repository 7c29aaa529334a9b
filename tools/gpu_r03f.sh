#!/bin/bash
# forward-only ring (4 slots) + two-pass network sum: tests, network line, network kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out/r03f
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --sampler network --step-factor 0.11 > $OUT/net.json 2> $OUT/net.err || { tail $OUT/net.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/net.json').read().strip().splitlines()[-1]); print('net', round(d['value'],1), round(d['ms_per_step'],3), d['accept_rate'], d.get('accept_rate_trajectories'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/nettrace -o run -- \
  python3 $R/bench.py --no-cpu-baseline --sampler network --steps 5 --warmup 2 --profile-iters 2 --step-factor 0.11 --accept-trajectories 0 > $OUT/nettrace.json 2> $OUT/nettrace.err || { echo "trace failed"; tail $OUT/nettrace.err; exit 1; }
grep -E "k_forward_fx|k_fused_grad_fx|k_net_sum|k_net_targets|k_residual_delta_sum" $OUT/nettrace/run_kernel_stats.csv | cut -d, -f1-4
