#!/bin/bash
# c3def bench lines: this tree vs rs-bann_amd/ab builds ($VARIANTS), gx scratch budgets ($BUDGETS MiB)
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r03k; mkdir -p $OUT
for a in base ${VARIANTS}; do
  LIBV=""; [ "$a" != base ] && LIBV=$R/rs-bann_amd/ab/librsbann_amd_$a.so
  for mb in ${BUDGETS:-8192}; do
    BANN_GX_SCRATCH_MB=$mb BANN_LIB=$LIBV timeout -k 10 300 python bench.py --config c3def --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --accept-trajectories 0 > $OUT/c3def_${a}_$mb.json 2> $OUT/c3def_${a}_$mb.err || { tail $OUT/c3def_${a}_$mb.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c3def_${a}_$mb.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c3def $a scratch $mb MiB', round(d['value'],3), round(d['ms_per_step'],1), 'k', round(r['kernel_ms'],1), 'acc', d['accept_rate'])"
  done
done
