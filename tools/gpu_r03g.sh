#!/bin/bash
# round profile of the current tree: C3 as the driver runs it, and C2
set -o pipefail
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
cd $R
bash tools/profile_round.sh r03g --steps 20 --warmup 5 > gpurun_out/r03g_c3.txt 2>&1 || { tail gpurun_out/r03g_c3.txt; exit 1; }
tail -12 gpurun_out/r03g_c3.txt
bash tools/profile_round.sh r03g_c2 --config c2 --steps 100 --warmup 10 > gpurun_out/r03g_c2.txt 2>&1 || { tail gpurun_out/r03g_c2.txt; exit 1; }
tail -8 gpurun_out/r03g_c2.txt
