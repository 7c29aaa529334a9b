#!/bin/bash
# SQ / TA / TCC counter passes of the C3 gradient kernel (and the forward-only pass)
# over tools/kbench.py, one rocprofv3 --pmc pass per counter group (kernel trace
# only), then tools/pmc_table.py: per-dispatch values, per tile and wave.
#   tools/pmc_fx.sh <tag> [kbench args]   (run from the repo root on the GPU box)
set -o pipefail
TAG=${1:-fx}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--branches 1000 --iters 3 --forward 2 $@"
run() { # name counters...
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o run -- \
    python3 $R/tools/kbench.py $ARGS > $OUT/$name.log 2>&1 || { echo "pass $name failed rc=$?"; tail -5 $OUT/$name.log; return 1; }
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT && \
run b SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS && \
run c SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES && \
run d SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_FLAT SQ_LEVEL_WAVES TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES && \
run e FETCH_SIZE && \
python3 $R/tools/pmc_table.py $OUT "$@"
