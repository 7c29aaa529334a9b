#!/bin/bash
# PMC passes over the kernel micro-benchmark (separate passes, kernel-trace only; no sys/runtime trace)
#   tools/pmc.sh <tag> [kbench args]      (env BANN_FUSED_VARIANT / BANN_LIB select the kernel)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
V=${1:-rx}; shift
ARGS="--iters 3 $@"
run() { # name counters...
  local name=$1; shift
  timeout -k 10 180 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/${V}_$name -o run -- python3 $R/tools/kbench.py $ARGS > $OUT/${V}_$name.log 2>&1 || { echo "pass $name failed rc=$?"; return 1; }
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU && \
run b SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE && \
run c FETCH_SIZE && \
run e SQ_LEVEL_WAVES SQ_ACCUM_PREV_HIRES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_COUNT
