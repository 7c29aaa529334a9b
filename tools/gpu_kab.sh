#!/bin/bash
# kernel A/B without a profiler: tools/kbench.py (back-to-back gradient launches, HIP events)
# for this tree's library ("base") and rs-bann_amd/ab/librsbann_amd_<v>.so, alternating, REPS times
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-kab}; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
for v in base ${VARIANTS}; do
  LIBV=""; [ "$v" != base ] && LIBV=$R/rs-bann_amd/ab/librsbann_amd_$v.so
  BANN_LIB=$LIBV timeout -k 10 200 python3 tools/kbench.py --branches ${NB:-1000} --iters ${ITERS:-30} --tag $v $KB > $OUT/${v}_$rep.txt 2>&1 || { tail -3 $OUT/${v}_$rep.txt; exit 1; }
  tail -1 $OUT/${v}_$rep.txt
done
done
