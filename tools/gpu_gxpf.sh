#!/bin/bash
# gx prefetch A/B: the GPU parity tests (this tree, then each variant library), then per-phase times
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-gxpf}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_base.log 2>&1 || { tail -30 $OUT/tests_base.log; exit 1; }
tail -1 $OUT/tests_base.log
for v in ${TESTV}; do
  BANN_LIB=$R/rs-bann_amd/ab/librsbann_amd_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_$v.log 2>&1 || { tail -30 $OUT/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/tests_$v.log)"
done
TAG=${TAG:-gxpf}/ph bash tools/gpu_gx_phases.sh
