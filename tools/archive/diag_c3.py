"""Diagnostic at C3 scale: forward-only predictions vs the gradient kernel's,
the target rebuild, and the acceptance of consecutive trajectories.
    python tools/diag_c3.py [branches]"""
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rs-bann_amd"))
sys.path.insert(0, ROOT)
from bench import init_branch_params  # noqa: E402
from bann import BannContext  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
n, m, widths = 50_000, 500, [4, 4, 1]
ctx = BannContext(0)
ctx.synthetic_genotypes(n, nb * m, seed=1000003)
for k in range(nb):
    ctx.add_branch(np.arange(k * m, (k + 1) * m, dtype=np.int32), widths, "tanh", "ridge_ard")
ctx.finalize(free_raw=True)
out_ss = 0.0
precs = []
for k in range(nb):
    pv, prec, ss = init_branch_params(np.random.default_rng(k), m, widths)
    ctx.set_params(k, pv)
    precs.append(prec)
    out_ss += ss
for k in range(nb):
    precs[k][len(widths) - 1] = np.array([nb / out_ss])
    ctx.set_precisions(k, np.concatenate(precs[k]).astype(np.float32))
fwd = ctx.predict_many(list(range(nb)))            # forward-only kernel
ctx.hmc_step(list(range(nb)), 0)                    # L = 0: the gradient kernel writes the predictions
grad = np.stack([ctx.predict(b) for b in range(0, nb, max(1, nb // 8))])   # cached rows (gradient kernel's)
sel = fwd[::max(1, nb // 8)]
print("fwd vs grad predictions: max |diff|", float(np.max(np.abs(sel - grad))), "max |f|", float(np.max(np.abs(sel))))
noise = np.random.default_rng(7).normal(0.0, math.sqrt(0.5), size=n).astype(np.float32)
ctx.residual_set(noise)
ctx.rebuild_targets(list(range(nb)))
r = [ctx.rss(b) for b in range(0, nb, max(1, nb // 8))]
print("rss against rebuilt targets", r[:3], "||noise||^2", float(np.sum(noise.astype(np.float64) ** 2)))
for t, L in enumerate([5, 2, 20, 20]):
    ctx.leapfrog_begin(list(range(nb)), L, 10.0, "izmailov", 1.0, seed=7 + t)
    ctx.leapfrog_steps(L)
    st, acc = ctx.leapfrog_end()
    print(f"trajectory {t}: L={L} accepted {acc}/{nb}, status counts {np.bincount(st, minlength=3)}")
    ctx.exchange_residual_device()
    ctx.rebuild_targets(list(range(nb)))
    r = ctx.residual_get()
    print("  residual sum sq", float(np.sum(r.astype(np.float64) ** 2)), "rss b0", ctx.rss(0))
ctx.close()
