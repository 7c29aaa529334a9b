#!/bin/bash
# Round profile of the bench command (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats of `bench.py` (the same command the driver runs)
#   2. separate PMC passes (kernel-trace only) for FETCH_SIZE and WRITE_SIZE
# then tools/summarize_profile.py writes profiles/<tag>_*.  Usage: tools/profile_round.sh r01 [bench args]
set -o pipefail
TAG=${1:-r01}; shift
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
  python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/bench_trace.json 2> $OUT/trace.err || { echo "trace pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o bench -- \
  python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 --profile-iters 2 "$@" > $OUT/bench_fetch.json 2> $OUT/fetch.err || { echo "fetch pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o bench -- \
  python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 --profile-iters 2 "$@" > $OUT/bench_write.json 2> $OUT/write.err || { echo "write pass failed"; exit 1; }
if [ -n "$PMC_MFMA" ]; then  # MFMA utilisation pass (SQ: 6 of 8 slots, GRBM: 2 of 2)
  timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $OUT/mfma -o bench -- \
    python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 --profile-iters 2 "$@" > $OUT/bench_mfma.json 2> $OUT/mfma.err || { echo "mfma pass failed"; exit 1; }
fi
cd $R && python3 tools/summarize_profile.py $TAG $OUT "$@"
