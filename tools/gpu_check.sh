#!/bin/bash
# parity suite + smoke + bench line (N=1): the round-end GPU tiers, in one call
set -o pipefail
mkdir -p gpurun_out/g
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g/pytest.txt 2>&1; rc=$?
tail -3 gpurun_out/g/pytest.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/g/pytest.txt | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/g/bench.json 2> gpurun_out/g/bench.err || { tail gpurun_out/g/bench.err; exit 1; }
cat gpurun_out/g/bench.json
