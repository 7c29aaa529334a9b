#!/bin/bash
# A/B of the wx kernel on a C5-shaped set (1000 branches x 125 SNPs, n = 100k, W = S = 32)
set -o pipefail
for r in 1 2; do for a in base $VARIANTS; do
  LIBV=""; [ "$a" != base ] && LIBV=rs-bann_amd/abl/librsbann_amd_abl$a.so
  BANN_LIB=$LIBV timeout -k 10 120 python tools/kbench.py --branches 1000 --n 100000 --m 125 --widths 32,32,1 --iters 5 --tag c5-$a || exit 1
done; done
