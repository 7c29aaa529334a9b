"""diagnostic: the device gradient_descent line search (emulated through the C
ABI in f32, as bann_net.cpp does) next to the oracle's, step by step, on one
lasso_ard branch: chosen step sizes and rss per probe."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "rs-bann_amd")]
import numpy as np
import bann_oracle as O
from helpers import f32_branch, x_std, build_context
from bann import BannContext

rng = np.random.default_rng(3)
n, m = 700, 64
g = O.synthetic_genotypes(rng, n, m)
br = f32_branch(O.random_branch(rng, m, [4, 4, 1], prior=sys.argv[1] if len(sys.argv) > 1 else "lasso_ard"))
y = rng.normal(size=n).astype(np.float32)
ctx = build_context(BannContext, g, [dict(snps=np.arange(m, dtype=np.int32), branch=br, y=y)])
mu, sd = ctx.genotype_stats()
X = x_std(g, mu, sd)
yd = y.astype(np.float64)
factor = np.float32(1e-4)

def dev_search(th, gv):
    def probe(s):
        ctx.set_params(0, (th + np.float32(s) * gv).astype(np.float32))
        return ctx.rss(0)
    s = np.float32(factor); prev = probe(s); tw = probe(2 * s)
    f = np.float32(2.0) if tw < prev else np.float32(0.5)
    s = s * f; cur = probe(s); trail = [prev, tw, cur]
    while cur < prev:
        prev = cur; s = s * f; cur = probe(s); trail.append(cur)
    return s / f, f, trail

def ora_search(ob, th, gv):
    def probe(s):
        ob.weights, ob.biases = O.load_param_vec(th + s * gv, m, [4, 4, 1])
        return O.rss(ob, X, yd)
    s = float(factor); prev = probe(s); tw = probe(2 * s)
    f = 2.0 if tw < prev else 0.5
    s *= f; cur = probe(s); trail = [prev, tw, cur]
    while cur < prev:
        prev = cur; s *= f; cur = probe(s); trail.append(cur)
    return s / f, f, trail

th_d = ctx.get_params(0)
ob = br.copy()
th_o = O.param_vec(ob.weights, ob.biases)
for k in range(10):
    ctx.set_params(0, th_d)
    gd, _ = ctx.log_density_gradient(0)
    ob.weights, ob.biases = O.load_param_vec(th_o, m, [4, 4, 1])
    gw, gb, _ = O.log_density_gradient(ob, X, yd)
    go = O.param_vec(gw, gb)
    sd_, fd, td = dev_search(th_d, gd)
    so, fo, to = ora_search(ob, th_o, go)
    print(k, "grad rel", float(np.linalg.norm(gd - go) / np.linalg.norm(go)), "step dev", float(sd_), fd, len(td),
          "ora", so, fo, len(to), "rss d/o", td[:3], to[:3], flush=True)
    th_d = (th_d + np.float32(sd_) * gd).astype(np.float32)
    th_o = th_o + so * go
    print("   theta rel", float(np.linalg.norm(th_d - th_o) / np.linalg.norm(th_o)))
