#!/bin/bash
# full GPU test suite, then bench lines for the given configs (default c3 c2); output under gpurun_out/b2
set -o pipefail
mkdir -p gpurun_out/b2
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b2/pytest.txt 2>&1; rc=$?
tail -3 gpurun_out/b2/pytest.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/b2/pytest.txt | head; exit 1; }
for c in ${CONFIGS:-c3 c2}; do
  timeout -k 10 300 python bench.py --config $c ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/b2/bench_$c.json 2> gpurun_out/b2/bench_$c.err || { tail -5 gpurun_out/b2/bench_$c.err; exit 1; }
  cat gpurun_out/b2/bench_$c.json
done
