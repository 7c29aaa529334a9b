#!/bin/bash
# state check of the tree: full GPU suite, smoke, C3 and C2 bench lines (output under gpurun_out/s)
set -o pipefail
mkdir -p gpurun_out/s
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s/pytest.txt 2>&1; rc=$?
tail -5 gpurun_out/s/pytest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s/smoke.txt 2>&1 || { cat gpurun_out/s/smoke.txt; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/s/bench_c3.json 2> gpurun_out/s/bench_c3.err || exit 1
cat gpurun_out/s/bench_c3.json
timeout -k 10 300 python bench.py --config c2 > gpurun_out/s/bench_c2.json 2> gpurun_out/s/bench_c2.err || exit 1
cat gpurun_out/s/bench_c2.json
