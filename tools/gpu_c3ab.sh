#!/bin/bash
# A/B of environment variants of a bench line, alternated on one box: VARIANTS="NAME=VAL[,NAME2=VAL2] ..."
# ("-" = defaults), BARGS = the bench arguments (default: the C3 line)
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-c3ab}; mkdir -p $OUT
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['value'],2), 'ms', round(d['ms_per_step'],4), 'k', round(r['kernel_ms'],4), 'upd', round(r['update_kernel_ms'],4), 'acc', d['accept_rate'], (d.get('accept_rate_trajectories') or {}).get('rate'))"; }
i=0
for rep in 1 2; do
  for v in ${VARIANTS:--}; do
    i=$((i+1))
    if [ "$v" = "-" ]; then E="env"; else E="env ${v//,/ }"; fi   # NAME=VAL,NAME2=VAL2
    $E timeout -k 10 300 python bench.py ${BARGS:---steps 20 --warmup 5} --no-cpu-baseline --no-network-check > $OUT/v$i.json 2> $OUT/v$i.err || { tail $OUT/v$i.err; exit 1; }
    echo -n "$v: "; j $OUT/v$i.json
  done
done
