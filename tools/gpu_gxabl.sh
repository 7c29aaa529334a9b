#!/bin/bash
# per-phase gx kernel times (one 40-branch group, c3def shape) for the default build and x3 ablations
set -o pipefail
R=$(pwd); mkdir -p gpurun_out/ga
cd /tmp && export TMPDIR=/tmp
for a in base ${VARIANTS:-1 2 4}; do
  LIBV=""; [ "$a" != base ] && LIBV=$R/rs-bann_amd/abl/librsbann_amd_gx$a.so
  BANN_LIB=$LIBV timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ga/$a -o k -- python3 $R/tools/kbench.py --branches 40 --widths 250,250,1 --iters 3 --tag gx$a > $R/gpurun_out/ga/$a.txt 2>&1 || { tail -3 $R/gpurun_out/ga/$a.txt; exit 1; }
  echo "== $a"; grep -h "k_gx" $R/gpurun_out/ga/$a/k_kernel_stats.csv | cut -d, -f1,4 | cut -c1-90
done
