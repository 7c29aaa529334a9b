#!/bin/bash
# per-phase stamps (FX_STAMPS builds from tools/build_ab.sh) of the C3 gradient launch, one kbench per variant
set -o pipefail
for v in $VARIANTS; do
  echo "== $v"
  BANN_STAMPS=1 BANN_LIB=$PWD/rs-bann_amd/ab/librsbann_amd_$v.so timeout -k 10 120 python3 tools/kbench.py --branches ${NB:-1000} --iters 20 2>&1 | grep -v "^$" || exit 1
done
