#!/bin/bash
# one GPU call: full parity suite, bench line, profile of the bench command (round tag $1)
set -o pipefail
TAG=${1:-r01c}
mkdir -p gpurun_out/g
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/g/pytest.txt 2>&1; rc=$?; echo pytest=$rc; tail -3 gpurun_out/g/pytest.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g/smoke.txt 2>&1 || { cat gpurun_out/g/smoke.txt; exit 1; }
cat gpurun_out/g/smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/g/bench.json 2> gpurun_out/g/bench.err || exit 1
cat gpurun_out/g/bench.json
bash tools/profile_round.sh $TAG > gpurun_out/g/profile.txt 2>&1 || { tail -5 gpurun_out/g/profile.txt; exit 1; }
