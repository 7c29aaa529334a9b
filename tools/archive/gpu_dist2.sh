#!/bin/bash
# the N-rank launcher rehearsed with 2 gloo ranks on one GPU (C3, C5): n_gpus 2, branch-shard x2
set -o pipefail
OUT=gpurun_out/dist2; mkdir -p $OUT
for cfg in c3 c5; do
  BANN_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > $OUT/$cfg.json 2> $OUT/$cfg.err || { tail -20 $OUT/$cfg.err; exit 1; }
  tail -1 $OUT/$cfg.json | cut -c1-420; grep network_check $OUT/$cfg.err | cut -c1-300
done
