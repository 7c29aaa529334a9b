#!/bin/bash
# round-6 GPU pass: PART=t the new / changed tests, then the whole -m gpu suite and smoke;
# PART=c (or BENCH=1 after the tests) the driver's C3 line and the network line (no profiles)
set -o pipefail
R=$(pwd); T=${TAG:-r06}; OUT=$R/gpurun_out/$T; mkdir -p $OUT
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; nc=d.get('network_check') or {}; print('$1', round(d['value'],2), 'ms', round(d['ms_per_step'],4), 'k', round(r['kernel_ms'],4), 'frac', round(r['frac'],4), 'acc', d['accept_rate'], (d.get('accept_rate_trajectories') or {}).get('rate'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'nc', nc.get('status'), nc.get('steps_per_s'), nc.get('forward_ms'), nc.get('gradient_ms'))"; }
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
if [ "${PART:-t}" = t ]; then
timeout -k 10 400 $PT tests/test_network_gpu.py tests/test_net_driver.py -m gpu > $OUT/tests_new.log 2>&1 || { tail -40 $OUT/tests_new.log; exit 1; }
tail -1 $OUT/tests_new.log
timeout -k 10 300 $PT tests/test_gpu_parity.py -m gpu -k "std_scaled or step_sizes or fxh" > $OUT/tests_new2.log 2>&1 || { tail -40 $OUT/tests_new2.log; exit 1; }
tail -1 $OUT/tests_new2.log
if [ -z "$QUICK" ]; then
timeout -k 10 700 $PT tests -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
fi
fi
if [ "${PART:-t}" = c ] || [ -n "$BENCH" ]; then
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/c3.json 2> $OUT/c3.err || { tail $OUT/c3.err; exit 1; }
j $OUT/c3.json
timeout -k 10 300 python bench.py --sampler network --steps 20 --warmup 2 --no-cpu-baseline --accept-trajectories 9 > $OUT/net.json 2> $OUT/net.err || { tail $OUT/net.err; exit 1; }
j $OUT/net.json
fi
