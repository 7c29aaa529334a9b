#!/bin/bash
# read-bandwidth probe + fx item-size sweep + stream-only / compute-only ablations (profiling)
set -o pipefail
mkdir -p gpurun_out/s
timeout -k 10 60 ./tools/probe_read > gpurun_out/s/probe.txt 2>&1 || { cat gpurun_out/s/probe.txt; exit 1; }
cat gpurun_out/s/probe.txt
for t in ${ITEMS:-2048 4096 8192 16384}; do
  BANN_TARGET_ITEMS=$t timeout -k 10 120 python tools/kbench.py --branches 1000 --tag items$t >> gpurun_out/s/kb.txt 2>&1 || exit 1
  BANN_TARGET_ITEMS=$t BANN_LIB=rs-bann_amd/abl/librsbann_amd_abl32.so timeout -k 10 120 python tools/kbench.py --branches 1000 --tag stream_items$t >> gpurun_out/s/kb.txt 2>&1 || exit 1
done
BANN_LIB=rs-bann_amd/abl/librsbann_amd_abl8.so timeout -k 10 120 python tools/kbench.py --branches 1000 --tag compute_only >> gpurun_out/s/kb.txt 2>&1 || exit 1
cat gpurun_out/s/kb.txt
