#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ts
for c in c3 c2; do for so in 1 0; do
  CFG=$c BANN_SOLO=$so timeout -k 10 120 python tools/time_solo.py 2>&1 | tail -3 || exit 1
done; done
cd /tmp && export TMPDIR=/tmp
CFG=c2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ts/tr -o ts -- python3 $GRAFT_REPO_ROOT/tools/time_solo.py > /dev/null 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/ts/tr -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-160 | head -12
