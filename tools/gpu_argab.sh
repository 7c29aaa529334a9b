#!/bin/bash
# bench-line A/B of two argument sets, alternated on one box: ARGS_A / ARGS_B, REPS pairs
set -o pipefail
OUT=gpurun_out/${TAG:-argab}; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-3}); do
  for v in A B; do
    eval "ARGS=\$ARGS_$v"
    timeout -k 10 300 python bench.py $ARGS > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { tail $OUT/${v}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/${v}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', $rep, round(d['value'],2), 'ms', round(d['ms_per_step'],4), 'k', round(r['kernel_ms'] or 0,4), 'upd', round(r['update_kernel_ms'] or 0,4))"
  done
done
