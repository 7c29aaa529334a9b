#!/bin/bash
# forward-only fx pass (network sampler's first launch) and the gradient launch: this tree vs $VARIANTS
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r03m; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for a in base ${VARIANTS}; do
  LIBV=""; [ "$a" != base ] && LIBV=$R/rs-bann_amd/ab/librsbann_amd_$a.so
  BANN_LIB=$LIBV timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$a -o k -- python3 $R/tools/kbench.py --branches 1000 --iters 20 --forward ${FWD:-10} --tag $a > $OUT/$a.txt 2>&1 || { tail -3 $OUT/$a.txt; exit 1; }
  echo "== $a"; grep -h '"tag"' $OUT/$a.txt; python3 -c "import csv;[print(r[\"Name\"][:30], r[\"Calls\"], round(float(r[\"AverageNs\"])/1e6,4), round(float(r[\"MinNs\"])/1e6,4)) for r in csv.DictReader(open(\"$OUT/$a/k_kernel_stats.csv\")) if \"fx\" in r[\"Name\"]]"
done
