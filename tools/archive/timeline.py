"""Kernel timeline of one trajectory from a rocprofv3 --kernel-trace CSV.

    python tools/timeline.py <kernel_trace.csv> [trajectory index (default 1 = the bench's timed one)] [--all]

A trajectory starts at a k_step_sizes launch (bann_leapfrog_begin / traj_prepare)
and ends at the last launch before the next one.  Prints per-kernel-name totals
(launches, busy ms, mean ms) and the idle time between launches, and with --all
every launch (offset, duration, gap to the previous launch's end)."""
import collections
import csv
import sys


def short(name):
    name = name.replace("void ", "")
    return name.split("(")[0][:60]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
want = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else 1
starts = [i for i, r in enumerate(rows) if "k_step_sizes" in r["Kernel_Name"]]
if want >= len(starts):
    sys.exit(f"only {len(starts)} trajectories in the trace")
lo = starts[want]
hi = starts[want + 1] if want + 1 < len(starts) else len(rows)
seg = rows[lo:hi]
t0 = int(seg[0]["Start_Timestamp"])
tot = collections.OrderedDict()
idle, prev_end = 0.0, None
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = 0.0 if prev_end is None else (s - prev_end) / 1e6
    idle += max(gap, 0.0)
    k = short(r["Kernel_Name"])
    n, busy = tot.get(k, (0, 0.0))
    tot[k] = (n + 1, busy + (e - s) / 1e6)
    if "--all" in sys.argv:
        print(f"{(s - t0) / 1e6:10.4f} ms  dur {(e - s) / 1e6:8.4f}  gap {gap:8.4f}  {k}")
    prev_end = e
span = (int(seg[-1]["End_Timestamp"]) - t0) / 1e6
print(f"trajectory {want}: {len(seg)} launches, span {span:.3f} ms, idle between launches {idle:.3f} ms")
for k, (n, busy) in tot.items():
    print(f"  {k:60s} {n:5d} launches  {busy:9.4f} ms  mean {busy / n:8.4f}")
