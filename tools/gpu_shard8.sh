#!/bin/bash
# rank 0's shard of an N = 2 / 4 / 8 job on this one GPU (no collective), plus a kernel trace at N = 8
set -o pipefail
mkdir -p gpurun_out/sh
R=$(pwd)
for e in 2 4 8; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --emulate-shard $e > gpurun_out/sh/e$e.json 2> gpurun_out/sh/e$e.err || { tail -3 gpurun_out/sh/e$e.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('shard', sys.argv[2], round(d['value'],1), round(d['ms_per_step'],4), 'grad', round(r['kernel_ms'],4), 'upd', round(r['update_kernel_ms'],4), 'frac', round(r['frac'],3))" gpurun_out/sh/e$e.json $e
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sh/trace -o sh -- python3 $R/bench.py --no-cpu-baseline --emulate-shard 8 > $R/gpurun_out/sh/trace.json 2> $R/gpurun_out/sh/trace.err || { tail -3 $R/gpurun_out/sh/trace.err; exit 1; }
head -8 $R/gpurun_out/sh/trace/sh_kernel_stats.csv | cut -c1-160
