#!/bin/bash
# bench-line A/B: this tree ("base") vs rs-bann_amd/ab/librsbann_amd_<v>.so for v in $VARIANTS (or, for
# v = env:NAME=VALUE, this tree's library under that environment variable), $REPS
# alternating reps of `bench.py $BARGS` (default: the driver's C3 command without the CPU baseline)
set -o pipefail
OUT=gpurun_out/${TAG:-bab}; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
for a in base ${VARIANTS}; do
  LIBV=""; EV=""
  case "$a" in base) ;; env:*) EV=${a#env:} ;; *) LIBV=$(pwd)/rs-bann_amd/ab/librsbann_amd_$a.so ;; esac
  env $EV BANN_LIB=$LIBV timeout -k 10 300 python bench.py ${BARGS:---steps 20 --warmup 5 --no-cpu-baseline} > $OUT/${a}_$rep.json 2> $OUT/${a}_$rep.err || { tail $OUT/${a}_$rep.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/${a}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$a', $rep, round(d['value'],2), 'ms', round(d['ms_per_step'],4), 'k', round(r['kernel_ms'],4), 'b2b', round(r['kernel_ms_back_to_back'] or 0,4), 'frac', round(r['frac'],4), 'acc', d['accept_rate'], (d.get('accept_rate_trajectories') or {}).get('rate'), 'fwd', round((d.get('network_timing') or {}).get('forward_ms') or 0, 4))"
done
done
