#!/bin/bash
# fx gradient launch back to back (C3, 1000 branches): this tree vs rs-bann_amd/ab builds ($VARIANTS), REPS rounds interleaved
set -o pipefail
for r in $(seq ${REPS:-2}); do
  for a in base $VARIANTS; do
    LIBV=""; [ "$a" != base ] && LIBV=rs-bann_amd/ab/librsbann_amd_$a.so
    BANN_LIB=$LIBV timeout -k 10 90 python tools/kbench.py --branches 1000 --iters ${ITERS:-40} --tag $a | grep '"tag"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['tag'], d['grad_ms'], d['alg_GBps'])" || exit 1
  done
done
