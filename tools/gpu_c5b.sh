#!/bin/bash
# C5: full-n wide parity, step-factor sweep for acceptance, counter list; output under gpurun_out/c5
set -o pipefail
mkdir -p gpurun_out/c5
timeout -k 10 300 python -u -m pytest tests -m gpu -k "c5_shape or wide" -v --timeout 200 --timeout-method thread > gpurun_out/c5/pytest.txt 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|assert" gpurun_out/c5/pytest.txt | head -20
[ $rc -eq 0 ] || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/c5/counters.txt 2>&1) || echo "counter list failed"
for f in ${FACTORS:-0.3 0.1 0.03}; do
  timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --step-factor $f --no-cpu-baseline > gpurun_out/c5/bench_$f.json 2> gpurun_out/c5/bench_$f.err || { tail -5 gpurun_out/c5/bench_$f.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c5/bench_$f.json')); print('$f', d['value'], d['accept_rate'], d['roofline']['kernel_ms'])"
done
