"""Writes tests/golden/sim_py_vectors.json from the reference's own numpy code.

Imports /root/reference/py-vis/sim.py (the reference's single-branch, no-hidden-
layer numpy model: tanh / leaky-relu predict, rss and the *full* rss
derivative d(rss)/d(w0), sim.py:42-54) and records its outputs on fixed
seeded inputs.  Only the resulting vectors are committed; the reference code
itself never travels.  Run in the build container:  python make_sim_py_vectors.py
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, "/root/reference/py-vis")
import sim  # noqa: E402  (reference module, build container only)

rng = np.random.default_rng(1234)
cases = []
for act in ("tanh", "lrelu"):
    for (n, m) in ((7, 3), (40, 11)):
        X = rng.normal(size=(n, m))
        y = rng.normal(size=n)
        w0 = rng.normal(scale=0.5, size=m)
        b0 = float(rng.normal(scale=0.3))
        w1 = float(rng.normal())
        p = sim.SingleBranchNoHiddenLayerParams(w0=w0, b0=b0, w1=w1)
        d = sim.Data(X=X, y=y)
        pred = getattr(sim, f"{act}_predict")(p, d)
        rss = getattr(sim, f"{act}_rss")(p, d)
        drss = getattr(sim, f"{act}_drssdw0")(p, d)
        cases.append(dict(act=act, n=n, m=m, X=X.tolist(), y=y.tolist(), w0=w0.tolist(), b0=b0,
                          w1=w1, predict=np.asarray(pred).tolist(), rss=float(rss),
                          drss_dw0_full=np.asarray(drss).tolist()))
here = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(here, "sim_py_vectors.json"), "w") as f:
    json.dump({"_source": "medical-genomics-group/rs-bann py-vis/sim.py:42-54 (full rss derivative, 2x the "
               "reference backpropagate convention)", "cases": cases}, f)
print("wrote", len(cases), "cases")
