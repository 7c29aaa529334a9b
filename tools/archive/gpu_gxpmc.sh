#!/bin/bash
# gx (c3def shape, one 40-branch group) PMC passes: FETCH_SIZE, WRITE_SIZE, MFMA busy (separate runs)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/gxpmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
KB="$R/tools/kbench.py --branches 40 --widths 250,250,1 --iters 2 --tag gxpmc"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o k -- python3 $KB > $O/trace.txt 2>&1 || { tail -3 $O/trace.txt; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o k -- python3 $KB > $O/fetch.txt 2>&1 || { tail -3 $O/fetch.txt; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o k -- python3 $KB > $O/write.txt 2>&1 || { tail -3 $O/write.txt; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/mfma -o k -- python3 $KB > $O/mfma.txt 2>&1 || { tail -3 $O/mfma.txt; exit 1; }
ls $O/*/
# the whole c3def bench line under the kernel trace (every phase of the 25-group evaluation)
cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench -o k -- python3 bench.py --config c3def --steps 4 --warmup 1 --no-cpu-baseline --accept-trajectories 0 > $O/bench.json 2> $O/bench.err || { tail -3 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-300
