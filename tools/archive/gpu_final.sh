#!/bin/bash
# end-of-round pass on one MI355X: GPU tests, smoke(), the round profile of the driver's
# command (kernel trace + PMC fetch/write), the driver's bench line with the CPU baseline,
# and the distributed launcher rehearsed with 2 gloo ranks on the one GPU (C3, C5)
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/final; mkdir -p $OUT
TAG=${TAG:-r03t}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json
bash tools/profile_round.sh $TAG --steps 20 --warmup 5 > $OUT/profile.log 2>&1 || { tail $OUT/profile.log; exit 1; }
tail -3 $OUT/profile.log
if [ -n "$C5" ]; then  # the C5 line and its round profile (wide kernel, MFMA pass)
  timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err || { tail $OUT/c5.err; exit 1; }
  tail -1 $OUT/c5.json | cut -c1-300
  PMC_MFMA=1 bash tools/profile_round.sh ${TAG}_c5 --config c5 --steps 10 --warmup 2 > $OUT/profile_c5.log 2>&1 || { tail $OUT/profile_c5.log; exit 1; }
  tail -3 $OUT/profile_c5.log
fi
if [ -n "$DIST" ]; then
  for cfg in c3 c5; do
    BANN_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > $OUT/dist2_$cfg.json 2> $OUT/dist2_$cfg.err || { tail -20 $OUT/dist2_$cfg.err; exit 1; }
    tail -1 $OUT/dist2_$cfg.json | cut -c1-400
  done
fi
