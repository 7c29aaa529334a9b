#!/bin/bash
# solo plans: fold + update in one launch (k_fold_update_solo) vs two; GPU tests first
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r03r; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for f in 1 0 1 0; do
  for g in ${GRAPH:-0}; do
    BANN_FOLD_MERGE=$f BANN_HMC_GRAPH=$g timeout -k 10 300 python bench.py --sampler sequential --steps 20 --warmup 0 --no-cpu-baseline > $OUT/seq_${f}_$g.json 2> $OUT/seq_${f}_$g.err || { tail $OUT/seq_${f}_$g.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/seq_${f}_$g.json').read().strip().splitlines()[-1]); print('seq merge $f graph $g', round(d['value'],2), round(d['ms_per_step'],2), 'acc', d['accept_rate'])"
  done
done
