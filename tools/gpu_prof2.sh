#!/bin/bash
# round profiles: C3 (fx) and C5 (wx, with the MFMA pass)
set -o pipefail
bash tools/profile_round.sh ${TAG:-r02e} > gpurun_out/prof_c3.txt 2>&1 || { tail -5 gpurun_out/prof_c3.txt; exit 1; }
tail -3 gpurun_out/prof_c3.txt
PMC_MFMA=1 bash tools/profile_round.sh ${TAG:-r02e}_c5 --config c5 > gpurun_out/prof_c5.txt 2>&1 || { tail -5 gpurun_out/prof_c5.txt; exit 1; }
tail -3 gpurun_out/prof_c5.txt
