#!/bin/bash
# kernel micro-benchmark over the fused-kernel variants and the ablation builds
# (make -C rs-bann_amd/csrc ablate first; profiling only)
set -e
ARGS="$@"
for v in mx pipe reg; do
  BANN_FUSED_VARIANT=$v timeout -k 10 120 python tools/kbench.py $ARGS --tag $v
done
for a in 1 2 4 3 7 8 15; do
  BANN_LIB=rs-bann_amd/abl/librsbann_amd_abl$a.so timeout -k 10 120 python tools/kbench.py $ARGS --tag mx_abl$a
done
