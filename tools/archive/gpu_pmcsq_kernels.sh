#!/bin/bash
# one SQ pass (issue, LDS, bank conflicts) over tools/kbench.py, summarised per kernel
#   KB="--branches 40 --widths 250,250,1 --iters 2" TAG=pmcgx bash tools/gpu_pmcsq_kernels.sh
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-pmck}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/sq -o run -- python3 $R/tools/kbench.py ${KB:---branches 40 --widths 250,250,1 --iters 2} > $OUT/sq.log 2>&1 || { echo "pass failed"; tail -5 $OUT/sq.log; exit 1; }
python3 $R/tools/pmc_by_kernel.py $(ls $OUT/sq/*counter_collection.csv | head -1) ${K:-} > $OUT/sq.txt && cat $OUT/sq.txt
