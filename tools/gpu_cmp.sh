#!/bin/bash
# A/B timing of the fused gradient kernel: default library vs ablation/experiment
# builds (rs-bann_amd/abl/librsbann_amd_abl<N>.so), interleaved, REPS rounds.
#   VARIANTS="512 1536" ITEMS=1024 ITERS=30 REPS=2 bash tools/gpu_cmp.sh
set -o pipefail
mkdir -p gpurun_out/cmp
ITEMS=${ITEMS:-1024}
ITERS=${ITERS:-30}
for r in $(seq ${REPS:-2}); do
  BANN_TARGET_ITEMS=$ITEMS timeout -k 10 60 python tools/kbench.py --branches 1000 --iters $ITERS --tag base || exit 1
  for a in $VARIANTS; do
    BANN_TARGET_ITEMS=$ITEMS BANN_LIB=rs-bann_amd/abl/librsbann_amd_abl$a.so \
      timeout -k 10 60 python tools/kbench.py --branches 1000 --iters $ITERS --tag v$a || exit 1
  done
done
