#!/bin/bash
# fx stamp builds (kbench, 1000 branches): cycles per phase and the shader clock
# (s_memtime / s_memrealtime over the tile loop) per variant
set -o pipefail
for a in ${VARIANTS:-16 131088 24}; do
  BANN_STAMPS=1 BANN_LIB=rs-bann_amd/abl/librsbann_amd_abl$a.so timeout -k 10 120 python tools/kbench.py --branches 1000 --tag abl$a || exit 1
done
