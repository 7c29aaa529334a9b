#!/bin/bash
# gx lazy head: (TESTS=1) GPU tests; per-phase times of one 40-branch c3def group and the
# c3def bench line, this tree vs the builds under rs-bann_amd/ab ($VARIANTS)
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-gxph}; mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
for a in base ${VARIANTS:-gxold}; do
  LIBV=""; [ "$a" != base ] && LIBV=$R/rs-bann_amd/ab/librsbann_amd_$a.so
  cd /tmp && export TMPDIR=/tmp
  BANN_LIB=$LIBV timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$a -o k -- python3 $R/tools/kbench.py --branches 40 --widths 250,250,1 --iters 3 --tag gx$a > $OUT/$a.txt 2>&1 || { tail -3 $OUT/$a.txt; exit 1; }
  echo "== $a"; python3 -c "import csv;[print(r[\"Name\"][:24], round(float(r[\"AverageNs\"])/1e6,3)) for r in csv.DictReader(open(\"$OUT/$a/k_kernel_stats.csv\")) if \"k_gx\" in r[\"Name\"]]"
  cd $R
  if [ -n "$BENCH" ]; then
    BANN_LIB=$LIBV timeout -k 10 300 python bench.py --config c3def --steps 4 --warmup 1 --no-cpu-baseline > $OUT/c3def_$a.json 2> $OUT/c3def_$a.err || { tail $OUT/c3def_$a.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c3def_$a.json').read().strip().splitlines()[-1]); print('c3def $a', round(d['value'],3), round(d['ms_per_step'],1), d['accept_rate'])"
  fi
done
