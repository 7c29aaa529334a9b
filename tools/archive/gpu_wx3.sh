#!/bin/bash
# wx3 (bf16-plane hidden GEMMs) on one MI355X: the wide parity tests, then the C5
# line on the plane path (default library and the A/B variant in $ALT) and on the
# exact f32 MFMA path (BANN_WX_EXACT=1)
set -o pipefail
OUT=gpurun_out/wx3; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wide or c5 or joint" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['value'],2), round(d['ms_per_step'],3), 'acc', d['accept_rate'], 'f', d['step_factor'], 'k', round(r['kernel_ms'],3), 'frac', round(r['frac'],4), r.get('bf16_pipe_frac'))"; }
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c5_planes.json 2> $OUT/c5_planes.err || { tail $OUT/c5_planes.err; exit 1; }
j $OUT/c5_planes.json
for a in $ALT; do
  BANN_LIB=rs-bann_amd/librsbann_amd_$a.so timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c5_$a.json 2> $OUT/c5_$a.err || { tail $OUT/c5_$a.err; exit 1; }
  j $OUT/c5_$a.json
done
if [ -n "$EXACT" ]; then
BANN_WX_EXACT=1 timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c5_exact.json 2> $OUT/c5_exact.err || { tail $OUT/c5_exact.err; exit 1; }
j $OUT/c5_exact.json
fi
