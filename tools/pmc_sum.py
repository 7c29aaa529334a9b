"""Summarise a rocprofv3 --pmc counter_collection.csv: per-dispatch sums of each
counter for kernels whose name contains argv[2], last dispatch, with ratios to
SQ_WAVE_CYCLES.   python tools/pmc_sum.py <csv> <kernel substring>"""
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if sys.argv[2] in r["Kernel_Name"]:
        by[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
d = sorted(by, key=int)[-1]
v = by[d]
W = v.get("SQ_WAVE_CYCLES", 0.0) or 1.0
for k, x in sorted(v.items()):
    print(f"{k:32s} {x:.4e}  {x / W:.3f}")
