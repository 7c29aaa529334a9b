"""Acceptance diagnostics for the C5 architecture (W = S = 32, m = 125, n = 100k; or M / N / WIDTH):
status counts and -H drift of bann_hmc_step trajectories at several Izmailov
factors, on a reduced branch count (same per-branch shape as bench.py --config c5)."""
import json, math, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rs-bann_amd"))
sys.path.insert(0, ROOT)
from bann import BannContext
from bench import init_branch_params

nb = int(os.environ.get("NB", 64))
m, n = int(os.environ.get("M", 125)), int(os.environ.get("N", 100_000))   # c3def: M=500 N=50000 WIDTH=250
W = [int(os.environ.get("WIDTH", 32))] * 2 + [1]
L = int(os.environ.get("L", 20))
ctx = BannContext(0)
ctx.synthetic_genotypes(n, nb * m, seed=3)
for k in range(nb):
    ctx.add_branch(np.arange(k * m, (k + 1) * m, dtype=np.int32), W, "tanh", "ridge_ard")
ctx.finalize(free_raw=True)
ps, precs, ss = [], [], 0.0
for k in range(nb):
    pv, prec, s = init_branch_params(np.random.default_rng(k), m, W)
    ps.append(pv); precs.append(prec); ss += s
for k in range(nb):
    precs[k][len(W) - 1] = np.array([nb / ss])
    ctx.set_params(k, ps[k]); ctx.set_precisions(k, np.concatenate(precs[k]).astype(np.float32))
preds = ctx.predict_many(list(range(nb)))
noise = np.random.default_rng(7).normal(0.0, max(float(np.std(preds.sum(0))), 1e-3), size=n)
for k in range(nb):
    ctx.set_target(k, (noise + preds[k]).astype(np.float32))
for c in [float(x) for x in os.environ.get("FACTORS", "0.3 0.1 0.03 0.01 0.003").split()]:
    for k in range(nb):
        ctx.set_params(k, ps[k])
    r = ctx.hmc_step(list(range(nb)), L, 10.0, "izmailov", c, seed=5)
    st = r["status"]
    tr = r["trace"]
    dh = tr[:, 1:] - tr[:, :1]
    fin = np.isfinite(dh)
    print(json.dumps(dict(factor=c, accepted=int((st == 0).sum()), rejected=int((st == 1).sum()),
                          early=int((st == 2).sum()), dH_step1_median=float(np.median(dh[:, 0])),
                          dH_last_median=float(np.median(np.where(fin, dh, np.nan)[:, -1])) if fin[:, -1].any() else None,
                          H0_median=float(np.median(tr[:, 0])))), flush=True)
# the packed leapfrog session (bench.py's path) at the same factors
for c in [float(x) for x in os.environ.get("FACTORS", "0.3 0.1 0.03 0.01 0.003").split()]:
    for k in range(nb):
        ctx.set_params(k, ps[k])
    ctx.leapfrog_begin(list(range(nb)), L, 10.0, "izmailov", c, seed=5)
    ctx.leapfrog_steps(L)
    st, acc = ctx.leapfrog_end()
    print(json.dumps(dict(session_factor=c, accepted=int((st == 0).sum()), rejected=int((st == 1).sum()),
                          early=int((st == 2).sum()))), flush=True)
