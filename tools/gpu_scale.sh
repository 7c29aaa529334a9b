#!/bin/bash
# parity suite, then the per-rank shard of the N-GPU bench emulated on one GPU
# (bench.py --emulate-shard N: rank 0's branches, no collective) and the N=1 line
set -o pipefail
mkdir -p gpurun_out/scale
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/scale/pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/scale/pytest.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/scale/pytest.txt | head -20; exit 1; }
for N in 8 4 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --emulate-shard $N ${BARGS:-} > gpurun_out/scale/shard$N.json 2> gpurun_out/scale/shard$N.err || { tail gpurun_out/scale/shard$N.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/scale/shard$N.json')); print($N, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['update_kernel_ms'])"
done
timeout -k 10 200 python bench.py --no-cpu-baseline ${BARGS:-} > gpurun_out/scale/n1.json 2> gpurun_out/scale/n1.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/scale/n1.json')); print(1, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
