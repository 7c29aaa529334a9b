#!/bin/bash
# run GPU tests selected by -k "$K" (no -x); summary lines + failures under gpurun_out/k
set -o pipefail
mkdir -p gpurun_out/k
timeout -k 10 ${LIMIT:-400} python -u -m pytest ${TESTS:-tests} -m gpu -k "$K" -v --timeout 120 --timeout-method thread \
  > gpurun_out/k/pytest.txt 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|assert" gpurun_out/k/pytest.txt | grep -v "^  " | head -80
exit $rc
