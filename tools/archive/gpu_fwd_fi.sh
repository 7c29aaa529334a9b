#!/bin/bash
# the forward-only pass: fi (individual-major image, kernels_fi.hip) vs the LDS forward (BANN_FWD_FI=0),
# both beside the gradient launch, in one kernel trace each (C3: 1000 branches x 500 SNPs, n = 50 000)
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-fwdfi}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for fi in 1 0; do
  BANN_FWD_FI=$fi timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fi$fi -o k -- python3 $R/tools/kbench.py --branches ${NB:-1000} --iters 20 --forward ${FWD:-20} --tag fi$fi > $OUT/fi$fi.txt 2>&1 || { tail -3 $OUT/fi$fi.txt; exit 1; }
  echo "== fi=$fi"; grep -h '"tag"' $OUT/fi$fi.txt; python3 -c "import csv;[print(r[\"Name\"][:40], r[\"Calls\"], round(float(r[\"AverageNs\"])/1e6,4), round(float(r[\"MinNs\"])/1e6,4)) for r in csv.DictReader(open(\"$OUT/fi$fi/k_kernel_stats.csv\")) if \"fx\" in r[\"Name\"] or \"fi\" in r[\"Name\"]]"
done
