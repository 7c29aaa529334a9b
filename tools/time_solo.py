"""Per-call latency of one-branch plans (the sequential driver's calls): hmc_step
of one branch at C2 / C3 shape, solo mode on (default) and off (BANN_SOLO=0)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rs-bann_amd"))
sys.path.insert(0, ROOT)
from bann import BannContext
from bench import init_branch_params

cfg = os.environ.get("CFG", "c3")
n, m, nb = {"c3": (50_000, 500, 16), "c2": (10_000, 2000, 16)}[cfg]
W = [4, 4, 1]
ctx = BannContext(0)
ctx.synthetic_genotypes(n, nb * m, seed=3)
for k in range(nb):
    ctx.add_branch(np.arange(k * m, (k + 1) * m, dtype=np.int32), W, "tanh", "ridge_ard")
ctx.finalize(free_raw=True)
for k in range(nb):
    pv, prec, s = init_branch_params(np.random.default_rng(k), m, W)
    prec[len(W) - 1] = np.array([1.0])
    ctx.set_params(k, pv)
    ctx.set_precisions(k, np.concatenate(prec).astype(np.float32))
    ctx.set_target(k, np.random.default_rng(k).normal(size=n).astype(np.float32))
L = 20
for rep in range(2):
    for what in ("grad", "hmc", "predict"):
        ctx.synchronize()
        t = time.perf_counter()
        for k in range(nb):
            if what == "grad":
                ctx.log_density_gradient(k)
            elif what == "hmc":
                ctx.hmc_step([k], L, 10.0, "izmailov", 1.0, seed=k)
            else:
                ctx.predict(k)
        ctx.synchronize()
        dt = (time.perf_counter() - t) / nb
        print(f"{cfg} solo={os.environ.get('BANN_SOLO', '1')} {what}: {dt * 1e3:.3f} ms per call"
              + (f" ({dt / L * 1e6:.1f} us per leapfrog step)" if what == "hmc" else ""), flush=True)
