# GPU tests (files in $SEL, default all; pytest -k expression in $K) in one pytest process
set -o pipefail
OUT=gpurun_out/${TAG:-t}; mkdir -p $OUT
timeout -k 10 ${TMO:-900} python -u -m pytest ${SEL:-tests} -m gpu ${K:+-k "$K"} -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" $OUT/tests.log | head -40; tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
