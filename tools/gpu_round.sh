#!/bin/bash
# one GPU call: parity tests, kernel micro-bench (+ ablations), bench line
set -o pipefail
mkdir -p gpurun_out/g
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/g/pytest.txt 2>&1; rc=$?; echo pytest=$rc; tail -3 gpurun_out/g/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python tools/kbench.py --branches 1000 --tag rx > gpurun_out/g/kbench.txt 2>&1 || exit 1
for a in ${ABL:-1 2 4 8 15}; do BANN_LIB=rs-bann_amd/abl/librsbann_amd_abl$a.so timeout -k 10 120 python tools/kbench.py --branches 1000 --tag rx_abl$a >> gpurun_out/g/kbench.txt 2>&1 || exit 1; done
cat gpurun_out/g/kbench.txt
timeout -k 10 400 python bench.py > gpurun_out/g/bench.json 2> gpurun_out/g/bench.err || exit 1
cat gpurun_out/g/bench.json
