#!/bin/bash
# A/B: default library vs variant builds on C3 (1000 branches) and C2 (64 x 2000 at n=10k), REPS rounds
set -o pipefail
mkdir -p gpurun_out/ab
for r in $(seq ${REPS:-2}); do
  for a in base $VARIANTS; do
    LIBV=""; [ "$a" != base ] && LIBV=rs-bann_amd/abl/librsbann_amd_abl$a.so
    BANN_LIB=$LIBV timeout -k 10 90 python tools/kbench.py --branches 1000 --iters ${ITERS:-30} --tag c3-$a || exit 1
    if [ -n "$C2" ]; then BANN_LIB=$LIBV timeout -k 10 90 python tools/kbench.py --branches 64 --n 10000 --m 2000 --iters ${ITERS:-30} --tag c2-$a || exit 1; fi
  done
done
