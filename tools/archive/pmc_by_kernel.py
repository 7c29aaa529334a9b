"""Per-kernel summary of a rocprofv3 --pmc counter_collection.csv: for every kernel
name containing argv[2] (default: all), the counters of its last dispatch and their
ratio to SQ_WAVE_CYCLES.   python tools/pmc_by_kernel.py <csv> [substring]"""
import collections, csv, sys

sub = sys.argv[2] if len(sys.argv) > 2 else ""
rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for r in rows:
    if sub in r["Kernel_Name"]:
        by[r["Kernel_Name"]][int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
for name, ds in by.items():
    v = ds[max(ds)]
    W = v.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    print(name.replace("void ", "").split("(")[0])
    for k, x in sorted(v.items()):
        print(f"  {k:32s} {x:.4e}  {x / W:.3f}")
