#!/bin/bash
# kernel timings of the default library and ablation libraries (LIBS="fabl1 fabl2"), shapes in KB
set -o pipefail
mkdir -p gpurun_out/kb
rm -f gpurun_out/kb/kb.txt
for lib in default $LIBS; do
  for s in ${KB:-64:10000:2000 64:50000:2000}; do
    IFS=: read b n m w <<< "$s"
    if [ $lib = default ]; then L=""; else L=rs-bann_amd/abl/librsbann_amd_$lib.so; fi
    BANN_LIB=$L timeout -k 10 120 python tools/kbench.py --branches $b --n $n --m $m ${w:+--widths $w} --iters ${ITERS:-20} --tag "$lib" >> gpurun_out/kb/kb.txt 2>&1 || { tail -5 gpurun_out/kb/kb.txt; exit 1; }
  done
done
cat gpurun_out/kb/kb.txt
