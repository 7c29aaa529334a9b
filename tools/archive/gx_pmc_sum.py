"""Summarise tools/gpu_gxpmc.sh (gx phases of one 40-branch c3def group): per kernel the
median duration, HBM fetch (FETCH_SIZE x 2, the gfx950 wide-read correction used for
the fx profiles too) and write bytes, and the matrix-pipe busy fraction
(SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), as tools/summarize_profile.py).
   python tools/gx_pmc_sum.py gpurun_out/gxpmc profiles/<tag>_c3def_pmc.md"""
import collections, csv, glob, statistics, sys

src, out = sys.argv[1], sys.argv[2]


def rows(sub, name):
    f = glob.glob(f"{src}/{sub}/**/*{name}", recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def short(n):
    return n.replace("void ", "").split("(")[0]


dur = collections.defaultdict(list)
for r in rows("trace", "kernel_trace.csv"):
    if "k_gx" in r["Kernel_Name"]:
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)


def counters(sub):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in rows(sub, "counter_collection.csv"):
        if "k_gx" not in r["Kernel_Name"]:
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        names[d] = short(r["Kernel_Name"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d, c in per.items():
        for k, v in c.items():
            agg[names[d]][k].append(v)
    return {n: {k: statistics.median(v) for k, v in c.items()} for n, c in agg.items()}


fe, wr, mf = counters("fetch"), counters("write"), counters("mfma")
lines = ["# gx PMC passes, c3def shape (one 40-branch group: n = 50 000, m = 500, W = S = 250)", "",
         "Command: tools/gpu_gxpmc.sh (kbench, separate --pmc runs per counter group); medians over the launches.", "",
         "| kernel | median ms | HBM fetch GB (x2) | write GB | TB/s | matrix pipes busy (per SIMD-cycle) |", "|---|---|---|---|---|---|"]
for n in sorted(dur, key=lambda k: -statistics.median(dur[k])):
    ms = statistics.median(dur[n])
    f = fe.get(n, {}).get("FETCH_SIZE", 0.0) * 1024 * 2 / 1e9
    w = wr.get(n, {}).get("WRITE_SIZE", 0.0) * 1024 / 1e9
    m = mf.get(n, {})
    busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (m.get("GRBM_GUI_ACTIVE", 1.0) / 8.0 * 1024) if m else 0.0
    lines.append(f"| {n} | {ms:.3f} | {f:.2f} | {w:.2f} | {(f + w) / ms:.2f} | {busy:.2f} |")
open(out, "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
