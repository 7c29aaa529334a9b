"""median / mean of the last K dispatches of each kernel family in rocprofv3 kernel traces:
    python tools/ab_trace_median.py <dir with <variant>_<rep>/k_kernel_trace.csv> [K]"""
import collections, csv, glob, os, statistics, sys
d = sys.argv[1]; K = int(sys.argv[2]) if len(sys.argv) > 2 else 15
rows = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*", "k_kernel_trace.csv"))):
    v = os.path.basename(os.path.dirname(f))
    ts = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        fam = "grad" if "k_fused_grad" in name else "fwd" if "k_forward" in name else "upd" if "k_update" in name else None
        if fam:
            ts[fam].append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    for fam, l in ts.items():
        l.sort()
        x = [t for _, t in l[-K:]]
        rows[(fam, v.rsplit("_", 1)[0])].append((statistics.median(x), statistics.mean(x)))
for (fam, v), l in sorted(rows.items()):
    print(f"{fam:5s} {v:12s} " + "  ".join(f"med {m:.4f} mean {a:.4f}" for m, a in l))
