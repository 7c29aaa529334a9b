#!/bin/bash
# round 3: sequential-driver kernel trace (graph replay), network step-factor sweep
set -o pipefail
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out/r03d
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/seq -o run -- \
  python3 $R/bench.py --no-cpu-baseline --sampler sequential --steps 20 --warmup 0 --profile-iters 2 > $OUT/seq.json 2> $OUT/seq.err || { echo "seq failed"; tail $OUT/seq.err; exit 1; }
cd $R
for f in 0.102 0.105 0.108 0.11; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --sampler network --step-factor $f > $OUT/net_$f.json 2> $OUT/net_$f.err || { tail $OUT/net_$f.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/net_$f.json').read().strip().splitlines()[-1]); print('net', $f, round(d['value'],1), d['accept_rate'])"
done
