#!/bin/bash
# gx phases (one 40-branch c3def group): dynamic instruction counts per kernel (one SQ pass)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/gxinst; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/sq -o k -- python3 $R/tools/kbench.py --branches 40 --widths 250,250,1 --iters 2 --tag gxinst > $O/sq.txt 2>&1 || { tail -3 $O/sq.txt; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob, collections
f=glob.glob('gpurun_out/gxinst/sq/**/*counter_collection.csv', recursive=True)[0]
per=collections.defaultdict(lambda: collections.defaultdict(float)); name={}
for r in csv.DictReader(open(f)):
    if 'k_gx' not in r['Kernel_Name']: continue
    d=r.get('Dispatch_Id') or r.get('Correlation_Id')
    per[d][r['Counter_Name']]+=float(r['Counter_Value']); name[d]=r['Kernel_Name'].replace('void ','').split('(')[0]
agg=collections.defaultdict(list)
for d,c in per.items(): agg[name[d]].append(c)
for n,L in agg.items():
    c=L[-1]; w=c['SQ_WAVES'] or 1
    print(n, 'waves', int(w), 'VALU/wave %.0f SALU/wave %.0f LDS/wave %.0f VMEM/wave %.0f MFMA-mops/wave %.0f' % (c['SQ_INSTS_VALU']/w, c['SQ_INSTS_SALU']/w, c['SQ_INSTS_LDS']/w, c['SQ_INSTS_VMEM_RD']/w, c['SQ_INSTS_VALU_MFMA_MOPS_BF16']/w))
PY
