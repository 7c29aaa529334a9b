#!/bin/bash
# quick iteration: parity subset + kernel timing (+ optional ablations via ABL="1 8")
set -o pipefail
mkdir -p gpurun_out/q
timeout -k 10 300 python -m pytest tests -m gpu -x -q ${PYK:--k "fx or delta or c3_shape or gradient_parity or hmc_step_parity"} > gpurun_out/q/pytest.txt 2>&1; rc=$?; echo pytest=$rc; tail -15 gpurun_out/q/pytest.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/kbench.py --branches 1000 --tag ${TAG:-fx} > gpurun_out/q/kbench.txt 2>&1 || { cat gpurun_out/q/kbench.txt; exit 1; }
for a in $ABL; do BANN_LIB=rs-bann_amd/abl/librsbann_amd_abl$a.so timeout -k 10 120 python tools/kbench.py --branches 1000 --tag abl$a >> gpurun_out/q/kbench.txt 2>&1 || exit 1; done
cat gpurun_out/q/kbench.txt
