#!/bin/bash
# SQ issue / stall / LDS-conflict counters of one gradient kernel over tools/kbench.py,
# one pass per counter set.  KB = kbench args, K = kernel-name substring, TAG = output dir
#   KB="--branches 500 --n 100000 --m 125 --widths 32,32,1" K=k_fused_grad_wx TAG=pmcwx bash tools/gpu_pmcsq.sh
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-pmcsq}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
KB="${KB:---branches 1000} --iters 3"
run() { local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o run -- python3 $R/tools/kbench.py $KB > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; return 1; }
  python3 $R/tools/pmc_sum.py $(ls $OUT/$name/*counter_collection.csv | head -1) ${K:-k_fused_grad} > $OUT/$name.txt && cat $OUT/$name.txt
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU && \
run b SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
