#!/bin/bash
# kernel timings for a list of "branches:n:m[:widths]" shapes (KB env), output under gpurun_out/kb
set -o pipefail
mkdir -p gpurun_out/kb
for s in ${KB:-64:10000:2000 64:50000:2000 256:10000:500 1000:50000:500}; do
  IFS=: read b n m w <<< "$s"
  timeout -k 10 120 python tools/kbench.py --branches $b --n $n --m $m ${w:+--widths $w} --iters ${ITERS:-20} --tag "$TAG" >> gpurun_out/kb/kb.txt 2>&1 || { tail -5 gpurun_out/kb/kb.txt; exit 1; }
done
cat gpurun_out/kb/kb.txt
