#!/bin/bash
# fused leapfrog update (fx): GPU tests, then C3 lines (driver's command) and the N = 8 shard, fused vs separate
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r03o; mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
j() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', round(d['value'],1), round(d['ms_per_step'],4), 'k', round(r['kernel_ms'],4), 'upd', round(r.get('update_kernel_ms',0),4), 'frac', round(r['frac'],4), 'acc', d['accept_rate'])"; }
for rep in ${REPS:-1}; do
for f in 1 0; do
  BANN_FUSE_UPD=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c3_$f.json 2> $OUT/c3_$f.err || { tail $OUT/c3_$f.err; exit 1; }
  j $OUT/c3_$f.json "c3 fuse=$f"
  BANN_FUSE_UPD=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --emulate-shard 8 > $OUT/s8_$f.json 2> $OUT/s8_$f.err || { tail $OUT/s8_$f.err; exit 1; }
  j $OUT/s8_$f.json "shard8 fuse=$f"
done
done
