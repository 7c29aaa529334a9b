#!/bin/bash
# update-kernel change: every GPU test, then kbench (one C3 branch, the C2 cohort) and the sequential line, this tree vs ab/old
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-updpre}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
TAG=${TAG:-updpre}/k1 VARIANTS=old REPS=2 NB=1 ITERS=200 KB="" bash tools/gpu_kab.sh || exit 1
TAG=${TAG:-updpre}/kc2 VARIANTS=old REPS=2 NB=64 ITERS=50 KB="--n 10000 --m 2000 --widths 4,4,1" bash tools/gpu_kab.sh || exit 1
TAG=${TAG:-updpre}/seq REPS=2 VARIANTS=old BARGS="--sampler sequential --steps 20 --warmup 0 --no-cpu-baseline" bash tools/gpu_bench_ab.sh
