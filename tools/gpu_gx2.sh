#!/bin/bash
# gx: parity subset, c3def acceptance sweep, c3def bench + trace (gpurun_out/gx)
set -o pipefail
mkdir -p gpurun_out/gx
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "layered or default_arch or gradient_parity or hmc_step_parity or momentum" > gpurun_out/gx/pytest.txt 2>&1 || { tail -30 gpurun_out/gx/pytest.txt; exit 1; }
tail -2 gpurun_out/gx/pytest.txt
NB=40 M=500 N=50000 WIDTH=250 L=20 FACTORS="0.3 0.1 0.05 0.02" timeout -k 10 300 python tools/c5_accept.py > gpurun_out/gx/accept.txt 2>&1 || { tail -5 gpurun_out/gx/accept.txt; exit 1; }
cat gpurun_out/gx/accept.txt
bash tools/gpu_gx.sh
