"""norm-relative gradient error per tensor of one tests/test_gpu_parity.py CONFIGS entry
against the oracle (GPU): python tools/wx_cfg_err.py <config index> [fused 0/1]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rs-bann_amd"))
import numpy as np
import conftest  # noqa: F401  (import paths)
import test_gpu_parity as T
import bann_oracle as O
from bann import BannContext as Context
ci = int(sys.argv[1]); fused = len(sys.argv) < 3 or sys.argv[2] == "1"
cfg = T.CONFIGS[ci]
rng, g, snps, br = T.make_problem(cfg, 100 + ci)
ctx = T.build_context(Context, g, [dict(snps=snps, branch=br, y=np.zeros(cfg["n"]))], fused=fused)
X = T.oracle_inputs(ctx, g, snps)
f = O.predict(br, X)
y = (f + rng.normal(scale=max(float(np.std(f)), 0.1), size=cfg["n"])).astype(np.float32).astype(np.float64)
ctx.set_target(0, y)
grad, rss = ctx.log_density_gradient(0)
ogw, ogb, orss = O.log_density_gradient(br, X, y)
gw, gb = T.layer_views(br, grad)
print(cfg, ctx.kernel_path(0), "W", [f"{T.norm_rel(gw[l], ogw[l]):.2e}" for l in range(br.num_layers)],
      "b", [f"{T.norm_rel(gb[l], ogb[l]):.2e}" for l in range(br.num_layers - 1)], "rss", rss, orss)
