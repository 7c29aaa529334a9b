#!/bin/bash
# sequential driver (bann_net_train, the reference's sweep order): bench lines with graph
# replay on (default) and off, then a kernel trace of one sweep (graph replay off: the
# profiler's kernel tracing does not follow graph launches)
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-seq}; mkdir -p $OUT
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', round(d['value'],3), 'ms', round(d['ms_per_step'],3), 'acc', d['accept_rate'])"; }
for v in 1 0; do
  BANN_HMC_GRAPH=$v timeout -k 10 400 python bench.py --sampler sequential --steps 20 --warmup 0 --no-cpu-baseline > $OUT/seq_g$v.json 2> $OUT/seq_g$v.err || { tail $OUT/seq_g$v.err; exit 1; }
  j $OUT/seq_g$v.json
done
cd /tmp && export TMPDIR=/tmp
BANN_HMC_GRAPH=0 timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/trace -o seq -- python3 $R/bench.py --sampler sequential --steps 20 --warmup 0 --no-cpu-baseline > $OUT/seq_trace.json 2> $OUT/seq_trace.err || { tail $OUT/seq_trace.err; exit 1; }
echo traced
