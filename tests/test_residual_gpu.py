"""The network residual on the device (include/bann.h "the network residual on
the device", bann_residual.hip) and the packed sweep's target rebuild.

  * the residual operations reproduce the reference's f32 element-wise order
    bitwise (initialize_stats net.rs:158-171, the partial-residual target
    279-280, the update 292-300, the output-bias shifts 319-332), with
    fixed-order f64 statistics;
  * a packed (Jacobi) sweep: two leapfrog sessions over every branch, each
    followed by bann_exchange_residual_device + bann_rebuild_targets, match the
    oracle's bookkeeping -- residual = residual - sum over accepted branches of
    f_b(theta_L) - f_b(theta_0), targets = residual + f_b -- and the second
    trajectory's gradients are the oracle's against the rebuilt targets.
"""
import numpy as np
import pytest

import bann_oracle as O
from helpers import f32_branch, norm_rel, x_std

pytestmark = pytest.mark.gpu

SHAPES = [(60, [4, 4, 1]), (100, [4, 4, 1]), (37, [3, 2, 1]), (128, [4, 4, 1]), (90, [4, 3, 1])]


def _setup(seed=4, n=1500):
    from bann import BannContext
    rng = np.random.default_rng(seed)
    M = sum(m for m, _ in SHAPES)
    g = O.synthetic_genotypes(rng, n, M)
    ctx = BannContext(0)
    ctx.upload_genotypes(g)
    brs, snps, off = [], [], 0
    for m, w in SHAPES:
        s = np.arange(off, off + m, dtype=np.int32)
        off += m
        ctx.add_branch(s, w, "tanh", "ridge_ard")
        brs.append(f32_branch(O.random_branch(rng, m, w)))
        snps.append(s)
    ctx.finalize()
    for b, br in enumerate(brs):
        ctx.set_params(b, O.param_vec(br.weights, br.biases))
        ctx.set_precisions(b, O.precision_vec(br))
    mu, sd = ctx.genotype_stats()
    X = [x_std(g[s], mu[s], sd[s]) for s in snps]
    f = sum(O.predict(br, x) for br, x in zip(brs, X))
    y = (f + rng.normal(scale=0.6, size=n)).astype(np.float32)
    return ctx, brs, X, y


def _with_params(br, pv):
    out = br.copy()
    out.weights, out.biases = O.load_param_vec(np.asarray(pv, np.float64), br.num_markers, br.layer_widths)
    return out


def test_residual_ops_match_reference_order():
    ctx, brs, X, y = _setup()
    nb = len(brs)
    preds = [ctx.predict(b) for b in range(nb)]
    bias = np.float32(0.37)
    s, q = ctx.residual_init(y, float(bias))
    r = y - bias                                  # f32, branch order (net.rs:160-166)
    for p in preds:
        r = r - p
    dev = ctx.residual_get()
    assert np.array_equal(dev, r)
    assert abs(s - float(np.sum(r, dtype=np.float64))) <= 1e-9 * max(1.0, abs(s)) + 1e-6
    assert abs(q - float(np.sum(r.astype(np.float64) ** 2))) <= 1e-9 * q
    # target of branch 2 = residual + f_2: its rss against the target is ||r||^2 up to rounding
    ctx.residual_to_target(2)
    assert abs(ctx.rss(2) - q) <= 1e-5 * q
    # new params for branch 2 -> residual = y_2 - f_2(new) (net.rs:295)
    pv = O.param_vec(brs[2].weights, brs[2].biases) * np.float32(0.9)
    ctx.set_params(2, pv)
    s2, q2 = ctx.residual_from_target(2)
    want = (r + preds[2]) - ctx.predict(2)
    assert np.array_equal(ctx.residual_get(), want)
    assert abs(q2 - float(np.sum(want.astype(np.float64) ** 2))) <= 1e-9 * q2
    # output bias shifts (net.rs:321, 332)
    s3, q3 = ctx.residual_shift(0.25)
    assert np.array_equal(ctx.residual_get(), want + np.float32(0.25))
    assert abs(s3 - float(np.sum((want + np.float32(0.25)).astype(np.float64)))) <= 1e-6 * max(1.0, abs(s3))
    ctx.close()


def test_jacobi_sweep_matches_oracle():
    ctx, brs, X, y = _setup(seed=8)
    nb = len(brs)
    all_b = list(range(nb))
    r = y.astype(np.float64) - sum(O.predict(br, x) for br, x in zip(brs, X))
    ctx.residual_set(r.astype(np.float32))
    ctx.rebuild_targets(all_b)
    theta = [O.param_vec(br.weights, br.biases) for br in brs]
    seen = set()
    for traj in range(2):
        if traj == 1:   # the rebuilt targets: every gradient is the oracle's against y_b = r + f_b
            for b in all_b:
                br = _with_params(brs[b], theta[b])
                yb = r + O.predict(br, X[b])
                gw, gb, _ = O.log_density_gradient(br, X[b], yb)
                g, _ = ctx.log_density_gradient(b)
                assert norm_rel(g, O.param_vec(gw, gb)) < 1e-5, b
        ctx.leapfrog_begin(all_b, 6, 10.0, "izmailov", 0.4, seed=11 + traj)
        ctx.leapfrog_steps(6)
        status, _ = ctx.leapfrog_end()
        seen.update(int(v) for v in status)
        new = [ctx.get_params(b) for b in all_b]
        for b in all_b:
            if status[b] != 0:
                assert np.array_equal(new[b], theta[b]), b   # rejected: restored
            else:
                r = r - (O.predict(_with_params(brs[b], new[b]), X[b]) - O.predict(_with_params(brs[b], theta[b]), X[b]))
        theta = [v.astype(np.float64) for v in new]
        ctx.exchange_residual_device()
        ctx.rebuild_targets(all_b)
        assert norm_rel(ctx.residual_get(), r) < 1e-5, traj
    ctx.close()
