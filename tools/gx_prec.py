"""Per-tensor norm-relative error of the gx gradient vs the float64 oracle, bf16x3
masked layer (default) vs BANN_GX_EXACT=1, on default-architecture branches."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("rs-bann_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import bann_oracle as O
from bann import BannContext
from helpers import build_context, f32_branch, layer_views, norm_rel, x_std

for n, m, w, seed in [(9000, 300, 150, 47), (9000, 300, 150, 48), (4000, 500, 250, 49), (20000, 200, 100, 50)]:
    rng = np.random.default_rng(seed)
    M = m + 7
    g = O.synthetic_genotypes(rng, n, M)
    snps = rng.permutation(M)[:m].astype(np.int32)
    br = f32_branch(O.random_branch(rng, m, [w, w, 1], prior="ridge_ard", act="tanh"))
    res = {}
    for ex in ("0", "1"):
        os.environ["BANN_GX_EXACT"] = ex
        ctx = build_context(BannContext, g, [dict(snps=snps, branch=br, y=np.zeros(n))])
        mu, sd = ctx.genotype_stats()
        X = x_std(g[snps], mu[snps], sd[snps])
        f = O.predict(br, X)
        y = (f + np.random.default_rng(seed).normal(scale=max(float(np.std(f)), 0.1), size=n)).astype(np.float32).astype(np.float64)
        ctx.set_target(0, y)
        grad, rss = ctx.log_density_gradient(0)
        ogw, ogb, orss = O.log_density_gradient(br, X, y)
        gw, gb = layer_views(br, grad)
        res[ex] = [norm_rel(gw[l], ogw[l]) for l in range(3)] + [norm_rel(gb[l], ogb[l]) for l in range(2)]
        ctx.close()
    print(n, m, w, "bf16x3:", " ".join(f"{v:.2e}" for v in res["0"]), "| exact:", " ".join(f"{v:.2e}" for v in res["1"]), flush=True)
