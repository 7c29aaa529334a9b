#!/bin/bash
# kernel A/B: this tree's library ("base") vs rs-bann_amd/ab/librsbann_amd_<v>.so for v in $VARIANTS,
# kbench (C3 by default: 1000 branches x 500 SNPs, n = 50 000) under a kernel trace: gradient, update and
# $FWD forward-only passes; KB: extra kbench args.  Repeated $REPS times in alternating order.
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-ab}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-1}); do
for a in base ${VARIANTS}; do
  LIBV=""; [ "$a" != base ] && LIBV=$R/rs-bann_amd/ab/librsbann_amd_$a.so
  d=$OUT/${a}_$rep
  BANN_LIB=$LIBV timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o k -- python3 $R/tools/kbench.py --branches ${NB:-1000} --iters 20 --forward ${FWD:-10} --tag $a $KB > $d.txt 2>&1 || { tail -3 $d.txt; exit 1; }
  echo "== $a rep $rep"; python3 -c "import csv;[print(r[\"Name\"][:34], r[\"Calls\"], round(float(r[\"AverageNs\"])/1e6,4), round(float(r[\"MinNs\"])/1e6,4)) for r in csv.DictReader(open(\"$d/k_kernel_stats.csv\")) if any(k in r[\"Name\"] for k in (\"fx\", \"fi<\", \"update\", \"wx\"))]"
done
done
