#!/bin/bash
# run the kernel micro-benchmark over kernel variants and ablation builds (profiling only)
set -e
ARGS="$@"
timeout -k 10 120 python tools/kbench.py $ARGS --tag pipe
BANN_FUSED_VARIANT=reg timeout -k 10 120 python tools/kbench.py $ARGS --tag reg
for a in 1 2 3; do
  BANN_LIB=rs-bann_amd/abl/librsbann_amd_abl$a.so timeout -k 10 120 python tools/kbench.py $ARGS --tag pipe_abl$a
done
