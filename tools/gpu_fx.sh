#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/fx
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/fx/pytest.txt 2>&1; rc=$?; echo pytest=$rc; tail -30 gpurun_out/fx/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python tools/kbench.py --branches 1000 --tag fx > gpurun_out/fx/kbench.txt 2>&1 || { cat gpurun_out/fx/kbench.txt; exit 1; }
for a in ${ABL:-1 2 4 8 15}; do BANN_LIB=rs-bann_amd/abl/librsbann_amd_abl$a.so timeout -k 10 120 python tools/kbench.py --branches 1000 --tag fx_abl$a >> gpurun_out/fx/kbench.txt 2>&1 || exit 1; done
cat gpurun_out/fx/kbench.txt
