#!/bin/bash
# C5: the f32 line and the bf16 hidden-GEMM line at step factors that keep its chain moving
set -o pipefail
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out/r03h
mkdir -p $OUT
cd $R
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['value'],2), round(d['ms_per_step'],3), 'acc', d['accept_rate'], 'f', d['step_factor'], 'k', round(r['kernel_ms'],3), 'frac', round(r['frac'],4))"; }
timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c5_f32.json 2> $OUT/c5_f32.err || { tail $OUT/c5_f32.err; exit 1; }
j $OUT/c5_f32.json
for f in 0.02 0.01; do
  timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline --hidden-bf16 --step-factor $f > $OUT/c5_bf16_$f.json 2> $OUT/c5_bf16_$f.err || { tail $OUT/c5_bf16_$f.err; exit 1; }
  j $OUT/c5_bf16_$f.json
done
