"""Per-branch-update host breakdown of the sequential driver from a rocprofv3 HIP API +
kernel trace (tools/gpu_seq_api.sh): branch updates are delimited by the second
k_residual_op of each update (the bias shift); over a mid-sweep window, the HIP API time
per function, the host time outside any HIP call, and the GPU busy / idle time."""
import csv, sys, collections
d = sys.argv[1]
api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in csv.DictReader(open(d + "/seq_hip_api_trace.csv"))]
ker = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(d + "/seq_kernel_trace.csv"))]
api.sort(); ker.sort()
res = [k for k in ker if k[2].startswith("k_residual_op")]
marks = [res[i][1] for i in range(1, len(res), 2)]  # end of each update's bias shift
lo, hi = len(marks) // 3, len(marks) // 3 + int(sys.argv[2] if len(sys.argv) > 2 else 50)
t0, t1 = marks[lo], marks[hi]
nb = hi - lo
fn = collections.defaultdict(lambda: [0, 0.0])
busy = 0
cur = t0
for s, e, f in api:
    if e <= t0 or s >= t1: continue
    s2, e2 = max(s, t0), min(e, t1)
    fn[f][0] += 1; fn[f][1] += (e2 - s2) / 1e3
    if e2 > cur:
        busy += (e2 - max(s2, cur)) / 1e3; cur = e2
span = (t1 - t0) / 1e3
kb = 0; curk = t0
kn = collections.defaultdict(lambda: [0, 0.0])
for s, e, f in ker:
    if e <= t0 or s >= t1: continue
    s2, e2 = max(s, t0), min(e, t1)
    if e2 > curk:
        kb += (e2 - max(s2, curk)) / 1e3; curk = e2
    kn[f.split("(")[0]][0] += 1; kn[f.split("(")[0]][1] += (e2 - s2) / 1e3
print(f"{nb} branch updates, {span / nb:.1f} us each: host inside HIP calls {busy / nb:.1f} us, outside {(span - busy) / nb:.1f} us; "
      f"GPU kernels busy {kb / nb:.1f} us, GPU idle {(span - kb) / nb:.1f} us")
print("HIP API per branch update (calls, us):")
for f, (c, t) in sorted(fn.items(), key=lambda x: -x[1][1]):
    print(f"  {f:36s} {c / nb:6.1f} {t / nb:8.1f}")
print("kernels per branch update (launches, us):")
for f, (c, t) in sorted(kn.items(), key=lambda x: -x[1][1])[:12]:
    print(f"  {f[:36]:36s} {c / nb:6.1f} {t / nb:8.1f}")
