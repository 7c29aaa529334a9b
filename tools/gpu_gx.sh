#!/bin/bash
# gx check on one MI355X: every GPU test, the c3def line, and one SQ pass per gx phase kernel
set -o pipefail
OUT=gpurun_out/gx; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python bench.py --config c3def --steps 10 --warmup 2 --no-cpu-baseline > $OUT/c3def.json 2> $OUT/c3def.err || { tail $OUT/c3def.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/c3def.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c3def', round(d['value'],3), round(d['ms_per_step'],1), 'acc', d.get('accept_rate'), 'k', round(r['kernel_ms'],1), 'frac', round(r['frac'],3))"
[ -n "$PMC" ] && K=k_gx TAG=gx/pmc bash tools/gpu_pmcsq_kernels.sh | grep -E "^k_|BANK|ACTIVE_INST_LDS|WAVE_CYCLES"
true
