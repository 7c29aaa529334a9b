#!/bin/bash
# GPU clock / power while the fx gradient launch runs back to back (kbench, 1000 branches): is it power-limited?
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/clk2; mkdir -p $OUT
(for i in $(seq 1 120); do amd-smi metric -g 0 -c -p --csv 2>/dev/null | tail -n +2; sleep 0.25; done) > $OUT/smi.csv 2>&1 &
SMI=$!
timeout -k 10 120 python3 tools/kbench.py --branches 1000 --iters 400 --tag clk > $OUT/kb.txt 2>&1
kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
cat $OUT/kb.txt | tail -2
head -3 $OUT/smi.csv; echo ...; sed -n '20,60p' $OUT/smi.csv | cut -c1-200
