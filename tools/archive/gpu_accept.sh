# acceptance of every bench line at the driver's L (20) and at L = 10 under the
# default step-factor rule (bench.py TUNED_FACTORS), plus the RCCL GPU test, the
# 1-rank RCCL network check and a 2-rank gloo rehearsal carrying network_check.
set -o pipefail
OUT=gpurun_out/${TAG:-acc}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_network_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/net_tests.log 2>&1 || { tail -30 $OUT/net_tests.log; exit 1; }
tail -1 $OUT/net_tests.log
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['value'],2), round(d['ms_per_step'],3), 'acc', d['accept_rate'], d.get('accept_rate_trajectories'), 'f', d['step_factor'], 'k', round(r['kernel_ms'],4), 'frac', round(r['frac'],4), 'nc', json.dumps(d.get('network_check')))"; }
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c3_rccl1.json 2> $OUT/c3_rccl1.err || { tail $OUT/c3_rccl1.err; exit 1; }
j $OUT/c3_rccl1.json
BANN_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c3_gloo2.json 2> $OUT/c3_gloo2.err || { tail -20 $OUT/c3_gloo2.err; exit 1; }
j $OUT/c3_gloo2.json
for L in ${LS:-10 20}; do
  for line in "--config c3" "--config c3 --sampler network" "--config c5" "--config c5 --hidden-bf16" ${C3DEF:+"--config c3def"}; do
    tag=$(echo "$line" | tr -d ' -')_L$L
    timeout -k 10 300 python bench.py $line --steps $L --warmup 2 --no-cpu-baseline > $OUT/$tag.json 2> $OUT/$tag.err || { tail $OUT/$tag.err; exit 1; }
    j $OUT/$tag.json
  done
done
