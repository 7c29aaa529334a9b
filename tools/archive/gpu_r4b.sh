#!/bin/bash
# round-4 pass b: GPU tests, then A/B lines (alternated on one box) for the fused update:
# the sequential driver (fused solo fold + update vs separate launches at the old split),
# C3 (one-split self-update vs the update launch), the N = 8 shard (last arriver vs launch)
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r4b}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
TAG=${TAG:-r4b}/seq VARIANTS="- BANN_FUSE_UPDATE=0,BANN_SOLO_TPW=1" BARGS="--sampler sequential --steps 20 --warmup 0" bash tools/gpu_c3ab.sh || exit 1
TAG=${TAG:-r4b}/c3 VARIANTS="- BANN_FUSE_UPDATE=0" bash tools/gpu_c3ab.sh || exit 1
TAG=${TAG:-r4b}/shard VARIANTS="- BANN_FUSE_UPDATE=1" BARGS="--emulate-shard 8 --steps 20 --warmup 5" bash tools/gpu_c3ab.sh || exit 1
