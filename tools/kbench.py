"""Kernel micro-benchmark: time the packed gradient launch (and the update
launch) for a synthetic C3-like branch set.  Library chosen by BANN_LIB.
  python tools/kbench.py --branches 250 --n 50000 --m 500"""
import argparse, json, math, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rs-bann_amd"))
from bann import BannContext

ap = argparse.ArgumentParser()
ap.add_argument("--branches", type=int, default=250)
ap.add_argument("--n", type=int, default=50000)
ap.add_argument("--m", type=int, default=500)
ap.add_argument("--widths", default="4,4,1")
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--tag", default="")
ap.add_argument("--forward", type=int, default=0, help="then K forward-only passes (bann_predict_many; time them in a kernel trace)")
a = ap.parse_args()
w = [int(x) for x in a.widths.split(",")]
ctx = BannContext(0)
ctx.synthetic_genotypes(a.n, a.branches * a.m, seed=5)
for b in range(a.branches):
    ctx.add_branch(np.arange(b * a.m, (b + 1) * a.m), w, "tanh", "ridge_ard")
ctx.finalize(free_raw=True)
rng = np.random.default_rng(0)
for b in range(a.branches):
    P = ctx.num_params(b)
    ctx.set_params(b, rng.normal(0, 1 / math.sqrt(a.m), P))
    ctx.set_precisions(b, np.ones(ctx.num_precisions(b)))
    ctx.set_target(b, rng.normal(size=a.n))
ctx.leapfrog_begin(list(range(a.branches)), 2, 10.0, "izmailov", 0.1, seed=1)
ctx.profile_session(2)
g, u = ctx.profile_session(a.iters)
xb = ((a.n + 3) // 4) * a.m * a.branches   # 2-bit genotypes (the .bed payload size)
print(json.dumps(dict(tag=a.tag, lib=os.environ.get("BANN_LIB", "default"), branches=a.branches, n=a.n, m=a.m,
                      path=ctx.kernel_path(0), grad_ms=round(g, 4), update_ms=round(u, 4),
                      alg_GBps=round((xb + 4 * a.n * a.branches) / g / 1e6, 1))), flush=True)
ctx.leapfrog_end()
for _ in range(a.forward):
    ctx.predict_many(list(range(a.branches)))
