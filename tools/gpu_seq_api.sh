#!/bin/bash
# sequential driver under a HIP runtime API + kernel + copy trace (no counters): where the
# host time between two branch updates goes (tools/seq_api_gaps.py summarizes)
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-seqapi}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BANN_HMC_GRAPH=${GRAPH:-1} timeout -k 10 500 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace -o seq -- python3 $R/bench.py --sampler sequential --steps 20 --warmup 0 --no-cpu-baseline > $OUT/seq_trace.json 2> $OUT/seq_trace.err || { tail $OUT/seq_trace.err; exit 1; }
ls -la $OUT/trace/*/ 2>/dev/null | head; ls -la $OUT/trace | head
