"""Counter table of the PMC passes of tools/pmc_fx.sh.

    python tools/pmc_table.py <pmc dir> [kbench args]

Every pass directory holds a rocprofv3 *counter_collection.csv; for each kernel
family (the gradient kernel, the forward-only pass, the update) this takes the
median over its dispatches of every counter and prints them with two
normalisations: per wave-cycle (SQ_WAVE_CYCLES; SQ cycle counters are in the same
quad-cycle unit) and per tile and wave (instruction counts / tiles, tiles =
branches x ceil(n / 64), each processed by one wave).  FETCH_SIZE is doubled
(gfx950 wide-read correction, MI355X_MICROARCH.md HBM).
"""
import argparse
import collections
import csv
import glob
import os
import statistics
import sys

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--branches", type=int, default=1000)
ap.add_argument("--n", type=int, default=50000)
ap.add_argument("--m", type=int, default=500)
a, _ = ap.parse_known_args()

FAMILIES = [("grad", "k_fused_grad"), ("forward", "k_forward"), ("update", "k_update")]
vals = collections.defaultdict(lambda: collections.defaultdict(list))  # family -> counter -> per-dispatch values
durs = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    for d, cs in per.items():
        fam = next((fa for fa, sub in FAMILIES if sub in names[d]), None)
        if fam is None:
            continue
        for c, v in cs.items():
            vals[fam][c].append(v)
for f in sorted(glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        fam = next((fa for fa, sub in FAMILIES if sub in r["Kernel_Name"]), None)
        if fam:
            durs[fam].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)

tiles = a.branches * ((a.n + 63) // 64)
print(f"# PMC table: {a.dir}\n\nworkload: {a.branches} branches x {a.m} SNPs, n = {a.n}: {tiles} tiles of 64 "
      "individuals per full launch (one wave per tile)\n")
for fam, _ in FAMILIES:
    if fam not in vals:
        continue
    med = {c: statistics.median(v) for c, v in vals[fam].items()}
    W = med.get("SQ_WAVE_CYCLES", 0.0)
    ms = statistics.median(durs[fam]) if durs[fam] else float("nan")
    print(f"## {fam}: {len(next(iter(vals[fam].values())))} dispatches per pass, median kernel time {ms:.4f} ms "
          f"(all passes)\n")
    print("| counter | median per dispatch | / SQ_WAVE_CYCLES | per tile-wave |")
    print("|---|---|---|---|")
    for c in sorted(med):
        v = med[c]
        if c == "FETCH_SIZE":
            v *= 2.0 * 1024  # KB -> bytes, x2 gfx950 correction
            print(f"| FETCH_SIZE x 2 (bytes) | {v:.4e} | | {v / tiles:.1f} B |")
            continue
        rw = f"{v / W:.3f}" if W and (c.startswith("SQ_WAIT") or c.startswith("SQ_ACTIVE") or c.startswith("SQ_BUSY")
                                      or c.endswith("CYCLES") or c.startswith("SQ_INST_LEVEL")
                                      or c.startswith("SQ_LEVEL")) else ""
        pt = f"{v / tiles:.1f}" if c.startswith("SQ_INSTS") else ""
        print(f"| {c} | {v:.4e} | {rw} | {pt} |")
    if "GRBM_GUI_ACTIVE" in med and ms == ms:
        print(f"\neffective clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time): "
              f"{med['GRBM_GUI_ACTIVE'] / 8 / (ms * 1e-3) / 1e9:.2f} GHz")
    print()
