#!/bin/bash
# update kernel block size A/B on the N = 8 shard and on C3
set -o pipefail
mkdir -p gpurun_out/sh
for r in 1 2; do for u in 0 1; do for e in 8 1; do
  BANN_UPD512=$u timeout -k 10 200 python bench.py --no-cpu-baseline --emulate-shard $e > gpurun_out/sh/u$u.json 2> gpurun_out/sh/u$u.err || { tail -3 gpurun_out/sh/u$u.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('upd512', sys.argv[2], 'shard', sys.argv[3], round(d['value'],1), round(d['ms_per_step'],4), 'upd', round(r['update_kernel_ms'],4), d['accept_rate'])" gpurun_out/sh/u$u.json $u $e
done; done; done
