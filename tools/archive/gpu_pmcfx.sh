#!/bin/bash
# counter list + SQ stall pass on the fx kernel (kbench, 1000 branches), output gpurun_out/pmc
set -o pipefail
R=$(pwd); mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
[ -s $R/gpurun_out/pmc/sq_names.txt ] || timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/pmc/counters.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" $R/gpurun_out/pmc/counters.txt | sort -u > $R/gpurun_out/pmc/sq_names.txt || true
timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_I8} --kernel-trace --output-format csv -d $R/gpurun_out/pmc/p1 -o p1 -- python3 $R/tools/kbench.py ${KBARGS:---branches 1000} --iters 3 > $R/gpurun_out/pmc/p1.txt 2>&1 || { tail -5 $R/gpurun_out/pmc/p1.txt; exit 1; }
ls $R/gpurun_out/pmc/p1
