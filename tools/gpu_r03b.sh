#!/bin/bash
# round 3: GPU tests of the new library paths, then bench lines (the driver's
# command, with / without launch timing) and the network sampler's step factor
set -o pipefail
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out/r03b
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -15 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/c3_$i.json 2> $OUT/c3_$i.err || { tail $OUT/c3_$i.err; exit 1; }
  tail -1 $OUT/c3_$i.json
done
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-launch-timing --no-cpu-baseline > $OUT/c3_nolt.json 2> $OUT/c3_nolt.err || exit 1
tail -1 $OUT/c3_nolt.json
for f in 0.05 0.1 0.2 0.4; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --sampler network --step-factor $f > $OUT/net_$f.json 2> $OUT/net_$f.err || { tail $OUT/net_$f.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/net_$f.json').read().strip().splitlines()[-1]); print('net', $f, d['value'], d['accept_rate'])"
done
