#!/bin/bash
# variant library ab/pk (update-kernel change): every GPU test against it, then kbench and the sequential line vs this tree
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-updpk}; mkdir -p $OUT
BANN_LIB=$R/rs-bann_amd/ab/librsbann_amd_pk.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
TAG=${TAG:-updpk}/k1 VARIANTS=pk REPS=2 NB=1 ITERS=200 KB="" bash tools/gpu_kab.sh || exit 1
TAG=${TAG:-updpk}/kc2 VARIANTS=pk REPS=2 NB=64 ITERS=50 KB="--n 10000 --m 2000 --widths 4,4,1" bash tools/gpu_kab.sh || exit 1
TAG=${TAG:-updpk}/seq REPS=2 VARIANTS=pk BARGS="--sampler sequential --steps 20 --warmup 0 --no-cpu-baseline" bash tools/gpu_bench_ab.sh
