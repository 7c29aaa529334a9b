"""Summarise tools/pmc.sh output: per-counter median over the full-size
launches of the fused gradient kernel.  usage: python tools/pmc_table.py <dir-prefix>"""
import csv, glob, statistics, sys
pre = sys.argv[1]
vals = {}
for f in glob.glob(pre + "_*/run_counter_collection.csv"):
    rows = list(csv.DictReader(open(f)))
    per = {}
    for r in rows:
        if "k_fused_grad" not in r["Kernel_Name"]:
            continue
        key = (r["Counter_Name"], r.get("Dispatch_Id"))
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
        per[("grid", r.get("Dispatch_Id"))] = int(r.get("Grid_Size", 0))
    gmax = max(v for (c, d), v in per.items() if c == "grid")
    disp = {d for (c, d), v in per.items() if c == "grid" and v == gmax}
    names = {c for (c, d) in per if c != "grid"}
    for c in names:
        vals[c] = statistics.median(per[(c, d)] for d in disp if (c, d) in per)
for k in sorted(vals):
    print(f"{k:28s} {vals[k]:.4g}")
