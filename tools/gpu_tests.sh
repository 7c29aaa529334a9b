#!/bin/bash
# run a subset of the GPU tests (default: all) with a per-test timeout; output under gpurun_out/t
#   TESTS="tests/test_net_driver.py" K="wide or parity" bash tools/gpu_tests.sh
set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 ${LIMIT:-400} python -u -m pytest ${TESTS:-tests} -m gpu ${K:+-k "$K"} -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/t/pytest.txt 2>&1
rc=$?
tail -40 gpurun_out/t/pytest.txt
exit $rc
