#!/bin/bash
# A/B of update-kernel builds on the bench's own step time: C3 (1000 branches) and the
# N = 8 shard (125 branches), default library vs rs-bann_amd/abl/librsbann_amd_abl<V>.so
set -o pipefail
mkdir -p gpurun_out/updab
for r in $(seq ${REPS:-2}); do
  for a in base $VARIANTS; do
    LIBV=""; [ "$a" != base ] && LIBV=rs-bann_amd/abl/librsbann_amd_abl$a.so
    for sh in 0 8; do
      BANN_LIB=$LIBV timeout -k 10 200 python bench.py --no-cpu-baseline --emulate-shard $sh > gpurun_out/updab/$a-$sh.json 2>/dev/null || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/updab/$a-$sh.json')); print('$a', $sh, round(d['value'],1), round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['update_kernel_ms'],4))"
    done
  done
done
