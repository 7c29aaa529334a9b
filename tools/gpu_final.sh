#!/bin/bash
# the round-end sequence: GPU tests, smoke(), the default bench line
set -o pipefail
mkdir -p gpurun_out/final
bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.txt 2>&1 || { tail -5 gpurun_out/final/smoke.txt; exit 1; }
tail -1 gpurun_out/final/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -5 gpurun_out/final/bench.err; exit 1; }
cat gpurun_out/final/bench.json
