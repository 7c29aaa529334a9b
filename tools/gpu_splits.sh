#!/bin/bash
# slot-aware fx split count vs the 1024-item target, at the per-rank shard sizes
set -o pipefail
for r in 1 2; do
for nb in 1000 500 250 125; do
  timeout -k 10 90 python tools/kbench.py --branches $nb --iters 30 --tag auto$nb || exit 1
  BANN_TARGET_ITEMS=1024 timeout -k 10 90 python tools/kbench.py --branches $nb --iters 30 --tag t1024_$nb || exit 1
done
done
