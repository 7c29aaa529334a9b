#!/bin/bash
# round refresh: bench lines (C3 default with the CPU baseline, C2, C5 f32 and bf16),
# then the round profiles (C3, C5 with the MFMA pass) under gpurun_out/prof_<TAG>*
set -o pipefail
mkdir -p gpurun_out/refresh
O=gpurun_out/refresh
timeout -k 10 400 python bench.py > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
cat $O/c3.json
timeout -k 10 300 python bench.py --config c2 > $O/c2.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
cat $O/c2.json
timeout -k 10 400 python bench.py --config c5 > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
cat $O/c5.json
timeout -k 10 300 python bench.py --config c5 --hidden-bf16 --no-cpu-baseline > $O/c5bf.json 2> $O/c5bf.err || { tail -5 $O/c5bf.err; exit 1; }
cat $O/c5bf.json
TAG=${TAG:-r02g} bash tools/gpu_prof2.sh
