#!/bin/bash
# read-bandwidth probe + stream-only / compute-only fx ablations (profiling)
set -o pipefail
mkdir -p gpurun_out/s
timeout -k 10 60 ./tools/probe_read > gpurun_out/s/probe.txt 2>&1 || { cat gpurun_out/s/probe.txt; exit 1; }
cat gpurun_out/s/probe.txt
for a in base ${VARIANTS:-32 8}; do
  LIBV=""; [ "$a" != base ] && LIBV=rs-bann_amd/abl/librsbann_amd_abl$a.so
  BANN_LIB=$LIBV timeout -k 10 120 python tools/kbench.py --branches 1000 --tag abl$a || exit 1
done
