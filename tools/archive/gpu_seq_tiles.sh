#!/bin/bash
# sequential driver (bann_net_train, C3, L = 20): solo tiles per wave sweep ($TILES), graph replay on/off
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r03n; mkdir -p $OUT
for t in ${TILES:-1 2 3 4}; do
  for g in ${GRAPH:-0}; do
    BANN_SOLO_TILES=$t BANN_HMC_GRAPH=$g timeout -k 10 300 python bench.py --sampler sequential --steps 20 --warmup 0 --no-cpu-baseline > $OUT/seq_${t}_$g.json 2> $OUT/seq_${t}_$g.err || { tail $OUT/seq_${t}_$g.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/seq_${t}_$g.json').read().strip().splitlines()[-1]); print('seq tiles $t graph $g', round(d['value'],2), round(d['ms_per_step'],2), 'acc', d['accept_rate'])"
  done
done
