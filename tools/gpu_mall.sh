#!/bin/bash
# does a gradient launch run faster once its genotype images fit the 256 MB Infinity Cache?
# kbench (back-to-back gradient launches on one theta) for a few branch counts, nt and cached LDS-DMA
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-mall}; mkdir -p $OUT
for nb in ${NBS:-16 32 64 128 1000}; do
for v in base nont; do
  LIBV=""; [ "$v" != base ] && LIBV=$R/rs-bann_amd/ab/librsbann_amd_$v.so
  BANN_LIB=$LIBV timeout -k 10 200 python3 tools/kbench.py --branches $nb --iters 20 --tag $v > $OUT/${v}_$nb.txt 2>&1 || { tail -3 $OUT/${v}_$nb.txt; exit 1; }
  tail -1 $OUT/${v}_$nb.txt
done
done
