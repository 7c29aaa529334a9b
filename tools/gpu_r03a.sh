#!/bin/bash
# round 3, first GPU pass: kernel timelines of the C3 timed trajectory (fixed
# per-trajectory cost) and of the sequential driver, and the C2 (fxl) round profile
set -o pipefail
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out/r03a
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/c3k20 -o run -- \
  python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 2 > $OUT/c3k20.json 2> $OUT/c3k20.err || { echo "c3k20 failed"; exit 1; }
cat $OUT/c3k20.json
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/seq -o run -- \
  python3 $R/bench.py --no-cpu-baseline --sampler sequential --steps 5 --warmup 0 > $OUT/seq.json 2> $OUT/seq.err || { echo "seq failed"; exit 1; }
cat $OUT/seq.json
cd $R && bash tools/profile_round.sh r03a_c2 --config c2
