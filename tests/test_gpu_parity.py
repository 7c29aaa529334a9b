"""GPU parity of the HIP hot path against the CPU oracle (and the reference KATs).

Every test calls through the C ABI (librsbann_amd.so via ctypes).  The oracle
(oracle/bann_oracle.py, float64) gets the SAME genotypes (downloaded from the
device), the same standardization constants and the f32-rounded parameters.

Tolerances (north_star: gradients and log-posterior within 1e-5 relative):
  * gradient tensors (per layer, weights and biases), predictions: norm-relative
    ||gpu - oracle|| / ||oracle|| <= 1e-5, on unsaturated synthetic inputs
    (standardized X, W ~ N(0, 1/m)).
  * rss, log density, -H: |gpu - oracle| <= 1e-5 * max(1, |oracle|).
  * reference KATs (saturated tanh): the per-tensor tolerances derived in
    tests/test_oracle_kats.py (1e-5, or the f32 cancellation bound ~1e-3 for the
    bias gradients).
"""
import json
import os

import numpy as np
import pytest

import bann_oracle as O
from helpers import build_context, f32_branch, layer_views, norm_rel, x_std

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))
TOL = 1e-5


@pytest.fixture(scope="module")
def Ctx():
    from bann import BannContext
    return BannContext


def scalar_close(a, b, tol=TOL):
    return abs(a - b) <= tol * max(1.0, abs(b))


# ---------------------------------------------------------------- KATs on GPU
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("prior", ["ridge_ard", "ridge_base", "lasso_ard", "lasso_base"])
def test_kat_gradient_gpu(Ctx, prior, fused):
    from test_oracle_kats import cancellation_tol
    X, y = O.kat_data()
    exp = KAT[prior]["ldg"]
    br = O.kat_branch(prior, exp["precision"])
    g = X.T.astype(np.int8)  # raw genotypes; mu = 0, sigma = 1 -> X_std == X
    ctx = build_context(Ctx, g, [dict(snps=[0, 1, 2], branch=br, y=y)], fused=fused,
                        stats=(np.zeros(3), np.ones(3)))
    assert ctx.kernel_path(0) == ("fused" if fused else "layered")
    grad, rss = ctx.log_density_gradient(0)
    gw, gb = layer_views(br, grad)
    for l in range(3):
        assert norm_rel(gw[l].reshape(-1, order="F"), exp["wrt_w"][l]) < TOL, (l, gw[l])
    for l in range(2):
        assert norm_rel(gb[l], exp["wrt_b"][l]) < cancellation_tol(br, X, l), (l, gb[l])
    assert scalar_close(rss, KAT["rss"])
    pred = ctx.predict(0)
    assert norm_rel(pred, KAT["forward_feed"]["out"]) < 1e-6
    ctx.close()


# ------------------------------------------------------ random-config parity
CONFIGS = [
    dict(n=1000, m=100, widths=[4, 4, 1], act="tanh", prior="ridge_ard"),
    dict(n=333, m=77, widths=[3, 2, 1], act="relu", prior="lasso_ard"),
    dict(n=500, m=130, widths=[4, 1], act="silu", prior="ridge_base"),
    dict(n=257, m=64, widths=[4, 4, 4, 1], act="leaky_relu", prior="lasso_base"),
    dict(n=100, m=5, widths=[2, 2, 1], act="identity", prior="std_normal"),
    dict(n=2000, m=500, widths=[4, 4, 1], act="tanh", prior="ridge_ard"),
    dict(n=700, m=1000, widths=[4, 4, 1], act="tanh", prior="ridge_ard"),
    dict(n=300, m=1100, widths=[4, 4, 1], act="tanh", prior="ridge_ard"),
    dict(n=400, m=60, widths=[8, 8, 1], act="tanh", prior="ridge_ard"),
    dict(n=1000, m=100, widths=[50, 50, 1], act="tanh", prior="ridge_ard"),
    dict(n=1, m=3, widths=[2, 1], act="tanh", prior="ridge_base"),
    # wide kernel (one hidden layer, W, S <= 32, m <= 128): C5's 32 x 32 at m = 125, ragged widths
    dict(n=1000, m=125, widths=[32, 32, 1], act="tanh", prior="ridge_ard"),
    dict(n=333, m=77, widths=[17, 9, 1], act="relu", prior="lasso_ard"),
    dict(n=500, m=128, widths=[5, 3, 1], act="silu", prior="ridge_base"),
    dict(n=257, m=40, widths=[32, 7, 1], act="leaky_relu", prior="lasso_base"),
    dict(n=100, m=64, widths=[12, 32, 1], act="identity", prior="std_normal"),
    dict(n=65, m=1, widths=[6, 6, 1], act="tanh", prior="ridge_ard"),
    # fxl (widths <= 4, 512 < m <= 4096: one wave per 512-marker block): C2's
    # 2 000-SNP branch at n = 10 000, full blocks, ragged blocks, 2 and 4 layers
    dict(n=10000, m=2000, widths=[4, 4, 1], act="tanh", prior="ridge_ard"),
    dict(n=1500, m=4096, widths=[4, 4, 1], act="relu", prior="lasso_ard"),
    dict(n=999, m=4000, widths=[3, 4, 1], act="silu", prior="ridge_base"),
    dict(n=300, m=577, widths=[4, 1], act="leaky_relu", prior="lasso_base"),
    dict(n=640, m=1536, widths=[2, 3, 4, 1], act="tanh", prior="ridge_ard"),
    dict(n=129, m=3000, widths=[4, 2, 1], act="identity", prior="std_normal"),
    # gx (layered MFMA GEMMs, any shape): the reference's default architecture
    # W = S = m_b / 2 (cli.rs:365-375), deep and ragged stacks, partial 64-tiles,
    # several row splits (n > 4096), a summary layer wider than one 256-thread pass
    dict(n=1200, m=300, widths=[150, 150, 1], act="tanh", prior="ridge_ard"),
    dict(n=700, m=500, widths=[250, 250, 1], act="relu", prior="lasso_ard"),
    dict(n=500, m=200, widths=[100, 70, 40, 1], act="silu", prior="ridge_base"),
    dict(n=4500, m=130, widths=[65, 65, 1], act="leaky_relu", prior="lasso_base"),
    dict(n=300, m=40, widths=[300, 1], act="tanh", prior="std_normal"),
    dict(n=9000, m=77, widths=[33, 5, 1], act="tanh", prior="ridge_ard"),
]


def expected_path(cfg, fused):
    """the kernel family bann_finalize picks (bann_api.hip)"""
    w, m = cfg["widths"], cfg["m"]
    if not fused:
        return "layered"
    if max(w) <= 4 and m <= 512 and len(w) <= 4:
        return "fused"
    if max(w) <= 4 and m <= 4096 and len(w) <= 4:
        return "fused_large"
    if len(w) == 3 and max(w) <= 32 and m <= 128:
        return "wide"
    return "layered"


def make_problem(cfg, seed):
    rng = np.random.default_rng(seed)
    n, m = cfg["n"], cfg["m"]
    M = m + 7
    g = O.synthetic_genotypes(rng, n, M)
    snps = rng.permutation(M)[:m].astype(np.int32)
    br = f32_branch(O.random_branch(rng, m, cfg["widths"], prior=cfg["prior"], act=cfg["act"]))
    return rng, g, snps, br


def oracle_inputs(ctx, g, snps):
    mu, sd = ctx.genotype_stats()
    X = x_std(g[snps], mu[snps], sd[snps])
    return X


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("ci", range(len(CONFIGS)))
def test_gradient_parity(Ctx, ci, fused):
    cfg = CONFIGS[ci]
    rng, g, snps, br = make_problem(cfg, 100 + ci)
    # y near the branch's own prediction (h^2 ~ 0.5 style residual)
    ctx0 = None
    ctx = build_context(Ctx, g, [dict(snps=snps, branch=br, y=np.zeros(cfg["n"]))], fused=fused)
    X = oracle_inputs(ctx, g, snps)
    f = O.predict(br, X)
    y = (f + rng.normal(scale=max(float(np.std(f)), 0.1), size=cfg["n"])).astype(np.float32).astype(np.float64)
    ctx.set_target(0, y)
    assert ctx.kernel_path(0) == expected_path(cfg, fused)
    grad, rss = ctx.log_density_gradient(0)
    ogw, ogb, orss = O.log_density_gradient(br, X, y)
    gw, gb = layer_views(br, grad)
    for l in range(br.num_layers):
        assert norm_rel(gw[l], ogw[l]) < TOL, ("W", l, norm_rel(gw[l], ogw[l]))
    for l in range(br.num_layers - 1):
        assert norm_rel(gb[l], ogb[l]) < TOL, ("b", l, norm_rel(gb[l], ogb[l]))
    assert scalar_close(rss, orss), (rss, orss)
    pred = ctx.predict(0)
    assert norm_rel(pred, f) < TOL
    ld = ctx.log_density(0, rss)
    assert scalar_close(ld, O.log_density(br, orss))
    p = rng.normal(size=br.num_params)
    assert scalar_close(ctx.neg_hamiltonian(0, p.astype(np.float32)),
                        O.log_density(br, orss) - 0.5 * float(np.sum(p.astype(np.float32).astype(np.float64) ** 2)))
    ctx.close()


def test_multi_branch_packed(Ctx):
    """Several branches of mixed shape/prior/path in one context (overlapping
    marker groups, as external.rs allows): every branch's gradient matches."""
    rng = np.random.default_rng(7)
    n, M = 777, 1500
    g = O.synthetic_genotypes(rng, n, M)
    shapes = [(500, [4, 4, 1], "tanh", "ridge_ard"), (64, [4, 1], "relu", "lasso_base"),
              (300, [2, 2, 1], "silu", "ridge_base"), (40, [6, 3, 1], "tanh", "lasso_ard"),
              (1024, [4, 4, 1], "tanh", "ridge_ard"), (200, [4, 4, 4, 1], "leaky_relu", "std_normal")]
    specs = []
    for m, w, a, p in shapes:
        snps = rng.choice(M, size=m, replace=False).astype(np.int32)
        br = f32_branch(O.random_branch(rng, m, w, prior=p, act=a))
        specs.append(dict(snps=snps, branch=br, y=rng.normal(size=n).astype(np.float32).astype(np.float64)))
    ctx = build_context(Ctx, g, specs)
    mu, sd = ctx.genotype_stats()
    for b, s in enumerate(specs):
        X = x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]])
        grad, rss = ctx.log_density_gradient(b)
        ogw, ogb, orss = O.log_density_gradient(s["branch"], X, s["y"])
        assert norm_rel(grad, O.param_vec(ogw, ogb)) < TOL, b
        assert scalar_close(rss, orss)
    ctx.close()


def test_predict_many_matches_predict(Ctx):
    rng = np.random.default_rng(17)
    n, m, nb = 901, 96, 6
    g = O.synthetic_genotypes(rng, n, nb * m)
    specs = [dict(snps=np.arange(b * m, (b + 1) * m, dtype=np.int32),
                  branch=f32_branch(O.random_branch(rng, m, [4, 4, 1] if b % 2 else [3, 1])),
                  y=rng.normal(size=n)) for b in range(nb)]
    ctx = build_context(Ctx, g, specs)
    order = [4, 0, 5, 2]
    many = ctx.predict_many(order)
    for i, b in enumerate(order):
        assert np.array_equal(many[i], ctx.predict(b))
    ctx.close()


def test_gradient_deterministic_and_split_invariant(Ctx):
    rng, g, snps, br = make_problem(dict(n=4000, m=500, widths=[4, 4, 1], act="tanh", prior="ridge_ard"), 3)
    y = rng.normal(size=4000)
    ctx = build_context(Ctx, g, [dict(snps=snps, branch=br, y=y)])
    g1, r1 = ctx.log_density_gradient(0)
    g2, r2 = ctx.log_density_gradient(0)
    assert np.array_equal(g1, g2) and r1 == r2  # fixed-order reductions: bitwise reproducible
    ctx.close()
    os.environ["BANN_TARGET_ITEMS"] = "1"      # one split instead of many (a one-branch plan
    os.environ["BANN_SOLO"] = "0"              # otherwise goes solo: ~one tile per wave)
    try:
        ctx = build_context(Ctx, g, [dict(snps=snps, branch=br, y=y)])
        g3, r3 = ctx.log_density_gradient(0)
    finally:
        del os.environ["BANN_TARGET_ITEMS"], os.environ["BANN_SOLO"]
    assert norm_rel(g3, g1) < 1e-6 and abs(r3 - r1) < 1e-6 * abs(r1)
    ctx.close()


# ----------------------------------------------------------------- HMC parity
@pytest.mark.parametrize("widths", [[4, 4, 1], [32, 32, 1]])
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("prior", ["ridge_ard", "lasso_base", "std_normal"])
def test_hmc_step_parity(Ctx, prior, fused, widths):
    """hmc_step (branch_sampler.rs:1192-1299) with injected momentum, step sizes
    and acceptance uniform: same trajectory, -H trace, status and end state
    (4-wide fused kernel, wide wx kernel, layered (gx) kernels)."""
    rng = np.random.default_rng(11)
    n, m, L = 600, 120, 6
    g = O.synthetic_genotypes(rng, n, m)
    snps = np.arange(m, dtype=np.int32)
    br = f32_branch(O.random_branch(rng, m, widths, prior=prior, act="tanh"))
    ctx = build_context(Ctx, g, [dict(snps=snps, branch=br, y=np.zeros(n))], fused=fused)
    X = oracle_inputs(ctx, g, snps)
    y = (O.predict(br, X) + rng.normal(scale=0.5, size=n)).astype(np.float32).astype(np.float64)
    ctx.set_target(0, y)
    ew, eb = O.izmailov_step_sizes(br, 0.5, L)
    eps = O.param_vec(ew, eb).astype(np.float32)
    p0 = rng.normal(size=br.num_params).astype(np.float32)
    res = ctx.hmc_step([0], L, 10.0, eps=eps, momentum=p0, u=[0.5])
    ow, ob = O.load_param_vec(eps.astype(np.float64), m, br.layer_widths)
    pw, pb = O.load_param_vec(p0.astype(np.float64), m, br.layer_widths)
    ob_ = br.copy()
    out = O.hmc_step(ob_, X, y, ow, ob, pw, pb, L, 10.0, 0.5)
    assert res["status"][0] == out["status"]
    tr = np.asarray(out["trace"])
    gt = res["trace"][0][: tr.size]
    assert np.all(np.abs(gt - tr) <= 1e-5 * np.maximum(1.0, np.abs(tr))), (gt, tr)
    final = ctx.get_params(0)
    assert norm_rel(final, O.param_vec(ob_.weights, ob_.biases)) < 1e-5
    assert res["uturn"][0] == out["u_turn_step"]
    ctx.close()


def test_c2_shape_hmc_and_packing(Ctx):
    """BASELINE config C2's branch shape (2 000 SNPs, W = S = 4, n = 10 000) on the
    fxl kernel: an HMC trajectory with injected draws matches the oracle, and a
    packed launch over fxl branches of 2, 4 and 8 wave blocks plus an fx branch
    gives every branch's oracle gradient; gradients are bitwise reproducible."""
    rng = np.random.default_rng(23)
    n, L = 10000, 5
    shapes = [(2000, [4, 4, 1]), (900, [4, 4, 1]), (4096, [2, 4, 1]), (300, [4, 4, 1])]
    M = sum(m for m, _ in shapes)
    g = O.synthetic_genotypes(rng, n, M)
    specs, off = [], 0
    for m, w in shapes:
        br = f32_branch(O.random_branch(rng, m, w))
        specs.append(dict(snps=np.arange(off, off + m, dtype=np.int32), branch=br, y=np.zeros(n)))
        off += m
    ctx = build_context(Ctx, g, specs)
    assert [ctx.kernel_path(b) for b in range(4)] == ["fused_large"] * 3 + ["fused"]
    mu, sd = ctx.genotype_stats()
    Xs = [x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]]) for s in specs]
    for b, s in enumerate(specs):
        s["y"] = (O.predict(s["branch"], Xs[b]) + rng.normal(scale=0.5, size=n)).astype(np.float32).astype(np.float64)
        ctx.set_target(b, s["y"])
    for b, s in enumerate(specs):
        grad, rss = ctx.log_density_gradient(b)
        ogw, ogb, orss = O.log_density_gradient(s["branch"], Xs[b], s["y"])
        assert norm_rel(grad, O.param_vec(ogw, ogb)) < TOL, b
        assert scalar_close(rss, orss), (b, rss, orss)
        grad2, _ = ctx.log_density_gradient(b)
        assert np.array_equal(grad, grad2)
    br = specs[0]["branch"]
    ew, eb = O.izmailov_step_sizes(br, 0.5, L)
    eps = O.param_vec(ew, eb).astype(np.float32)
    p0 = rng.normal(size=br.num_params).astype(np.float32)
    res = ctx.hmc_step([0], L, 10.0, eps=eps, momentum=p0, u=[0.5])
    ow, ob = O.load_param_vec(eps.astype(np.float64), 2000, br.layer_widths)
    pw, pb = O.load_param_vec(p0.astype(np.float64), 2000, br.layer_widths)
    ob_ = br.copy()
    out = O.hmc_step(ob_, Xs[0], specs[0]["y"], ow, ob, pw, pb, L, 10.0, 0.5)
    assert res["status"][0] == out["status"]
    tr = np.asarray(out["trace"])
    gt = res["trace"][0][: tr.size]
    assert np.all(np.abs(gt - tr) <= 1e-5 * np.maximum(1.0, np.abs(tr))), (gt, tr)
    assert norm_rel(ctx.get_params(0), O.param_vec(ob_.weights, ob_.biases)) < 1e-5
    ctx.close()


def test_hmc_early_rejection_restores(Ctx):
    """|dH| > max_hamiltonian_error -> RejectedEarly and initial params restored (1264-1279)."""
    rng = np.random.default_rng(5)
    n, m = 300, 64
    g = O.synthetic_genotypes(rng, n, m)
    br = f32_branch(O.random_branch(rng, m, [4, 4, 1]))
    ctx = build_context(Ctx, g, [dict(snps=np.arange(m), branch=br, y=rng.normal(size=n))])
    before = ctx.get_params(0)
    eps = np.full(br.num_params, 5.0, np.float32)   # absurd step sizes
    res = ctx.hmc_step([0], 4, 0.1, eps=eps, momentum=np.ones(br.num_params, np.float32), u=[0.0])
    assert res["status"][0] == 2
    assert np.array_equal(ctx.get_params(0), before)
    ctx.close()


def test_hmc_packed_equals_individual(Ctx):
    """Packing branches into one launch does not change any branch's trajectory."""
    rng = np.random.default_rng(9)
    n, M = 400, 300
    g = O.synthetic_genotypes(rng, n, M)
    specs = []
    for k in range(4):
        snps = rng.choice(M, size=100, replace=False).astype(np.int32)
        br = f32_branch(O.random_branch(rng, 100, [4, 4, 1]))
        specs.append(dict(snps=snps, branch=br, y=rng.normal(size=n)))
    P = specs[0]["branch"].num_params
    eps = np.concatenate([O.param_vec(*O.izmailov_step_sizes(s["branch"], 0.3, 5)) for s in specs]).astype(np.float32)
    p0 = rng.normal(size=4 * P).astype(np.float32)
    u = np.array([0.3, 0.6, 0.9, 0.1], np.float32)
    ctx = build_context(Ctx, g, specs)
    r_all = ctx.hmc_step([0, 1, 2, 3], 5, 10.0, eps=eps, momentum=p0, u=u)
    params_all = [ctx.get_params(b) for b in range(4)]
    ctx.close()
    for b in range(4):
        ctx = build_context(Ctx, g, specs)
        r1 = ctx.hmc_step([b], 5, 10.0, eps=eps[b * P:(b + 1) * P], momentum=p0[b * P:(b + 1) * P], u=u[b:b + 1])
        assert r1["status"][0] == r_all["status"][b]
        assert np.array_equal(ctx.get_params(b), params_all[b])
        assert np.array_equal(r1["trace"][0], r_all["trace"][b])
        ctx.close()


@pytest.mark.parametrize("mode", ["izmailov", "uniform"])
def test_device_step_sizes_match_oracle(Ctx, mode):
    """Izmailov / uniform step sizes formed on the device equal the oracle's
    (izmailov_step_sizes of the five priors, branch_sampler.rs:706-732)."""
    rng = np.random.default_rng(31)
    n, m = 128, 40
    priors = ["ridge_ard", "ridge_base", "lasso_ard", "lasso_base", "std_normal"]
    g = O.synthetic_genotypes(rng, n, m * len(priors))
    specs = [dict(snps=np.arange(k * m, (k + 1) * m, dtype=np.int32),
                  branch=f32_branch(O.random_branch(rng, m, [4, 3, 1], prior=p)), y=rng.normal(size=n))
             for k, p in enumerate(priors)]
    ctx = build_context(Ctx, g, specs)
    L, c = 7, 0.37
    ctx.leapfrog_begin(list(range(len(priors))), L, 10.0, mode, c, seed=1)
    ctx.leapfrog_end()
    for k, s in enumerate(specs):
        got = ctx.get_step_sizes(k)
        if mode == "uniform":
            ref = np.full(got.size, np.float32(c))
        else:
            ref = O.param_vec(*O.izmailov_step_sizes(s["branch"], c, L)).astype(np.float32)
        assert np.allclose(got, ref, rtol=2e-7, atol=0), (priors[k], np.max(np.abs(got / ref - 1)))
    ctx.close()


def test_std_scaled_step_sizes_match_oracle(Ctx):
    """StepSizeMode::StdScaled (branch_sampler.rs:1213): c * sqrt(1 / lambda_l) per weight
    layer and c * (1 / sqrt(lambda_b)) per bias for RidgeBase / LassoBase / StdNormal
    (ridge_base.rs:52-82, lasso_base.rs:53-82, std_normal_branch.rs:51-80) equal the oracle's
    f32 restatement to 2e-7; the ARD priors, whose reference vectors are empty
    (ridge_ard.rs:56-68, lasso_ard.rs:62-74), are refused."""
    from bann import BannError
    rng = np.random.default_rng(32)
    n, m = 128, 40
    priors = ["ridge_base", "lasso_base", "std_normal", "ridge_ard", "lasso_ard"]
    g = O.synthetic_genotypes(rng, n, m * len(priors))
    specs = [dict(snps=np.arange(k * m, (k + 1) * m, dtype=np.int32),
                  branch=f32_branch(O.random_branch(rng, m, [4, 3, 1], prior=p)), y=rng.normal(size=n))
             for k, p in enumerate(priors)]
    ctx = build_context(Ctx, g, specs)
    L, c = 7, 0.37
    ctx.leapfrog_begin([0, 1, 2], L, 10.0, "std_scaled", c, seed=1)
    ctx.leapfrog_end()
    for k in range(3):
        got = ctx.get_step_sizes(k)
        ref = O.param_vec(*O.std_scaled_step_sizes(specs[k]["branch"], c)).astype(np.float32)
        assert np.allclose(got, ref, rtol=2e-7, atol=0), (priors[k], np.max(np.abs(got / ref - 1)))
    for k in (3, 4):
        with pytest.raises(BannError, match="ARD"):
            ctx.hmc_step([k], L, 10.0, step_mode="std_scaled", step_factor=c, seed=2)
        with pytest.raises(ValueError):
            O.std_scaled_step_sizes(specs[k]["branch"], c)
    ctx.close()


@pytest.mark.parametrize("prior", ["ridge_base", "lasso_base", "std_normal"])
def test_hmc_step_std_scaled_matches_oracle(Ctx, prior):
    """A whole hmc_step trajectory in StdScaled mode (the step sizes formed by the library,
    momentum and uniform injected) reproduces the oracle's -H trace, status and end state."""
    rng = np.random.default_rng(33)
    n, m, L, c = 400, 96, 8, 0.02
    g = O.synthetic_genotypes(rng, n, m)
    br = f32_branch(O.random_branch(rng, m, [4, 4, 1], prior=prior))
    ctx = build_context(Ctx, g, [dict(snps=np.arange(m, dtype=np.int32), branch=br, y=np.zeros(n))])
    mu, sd = ctx.genotype_stats()
    X = x_std(g, mu, sd)
    y = (O.predict(br, X) + rng.normal(scale=0.5, size=n)).astype(np.float32).astype(np.float64)
    ctx.set_target(0, y)
    p0 = rng.normal(size=br.num_params).astype(np.float32)
    res = ctx.hmc_step([0], L, 10.0, step_mode="std_scaled", step_factor=c, momentum=p0, u=[0.5])
    ew, eb = O.std_scaled_step_sizes(br, c)
    ew = [e.astype(np.float64) for e in ew]
    eb = [e.astype(np.float64) for e in eb]
    pw, pb = O.load_param_vec(p0.astype(np.float64), m, br.layer_widths)
    ob_ = br.copy()
    out = O.hmc_step(ob_, X, y, ew, eb, pw, pb, L, 10.0, 0.5)
    assert res["status"][0] == out["status"]
    tr = np.asarray(out["trace"])
    gt = res["trace"][0][: tr.size]
    assert np.all(np.abs(gt - tr) <= 1e-5 * np.maximum(1.0, np.abs(tr))), (gt, tr)
    assert norm_rel(ctx.get_params(0), O.param_vec(ob_.weights, ob_.biases)) < 1e-5
    ctx.close()


def test_device_momentum_moments(Ctx):
    """k_sample_momentum (sample_momentum, branch_sampler.rs:594-609: p ~ N(0, 1)):
    the device momenta are recovered from the first recorded position step of a
    trajectory with injected eps = 1e-2 (theta_1 = theta_0 + eps (p + eps/2
    ldg(theta_0))) and must look standard normal -- mean, variance, kurtosis,
    KS distance, no lag-1 or cross-branch correlation; the same seed gives the same
    draws, another seed different ones."""
    from scipy import stats
    rng = np.random.default_rng(41)
    n, m, nb = 300, 256, 8
    g = O.synthetic_genotypes(rng, n, nb * m)
    specs = [dict(snps=np.arange(b * m, (b + 1) * m, dtype=np.int32),
                  branch=f32_branch(O.random_branch(rng, m, [4, 4, 1])), y=rng.normal(size=n)) for b in range(nb)]
    ctx = build_context(Ctx, g, specs)
    P = ctx.num_params(0)
    e = 1e-2
    ctx.set_trajectory_recording(True)

    def draw(seed):
        th0 = [ctx.get_params(b).astype(np.float64) for b in range(nb)]
        ldg0 = [ctx.log_density_gradient(b)[0].astype(np.float64) for b in range(nb)]
        ctx.hmc_step(list(range(nb)), 1, 1e9, eps=np.full(nb * P, e, np.float32), seed=seed, u=np.zeros(nb))
        ps = []
        for b in range(nb):
            th1 = ctx.get_trajectory(b)["params"][0].astype(np.float64)
            ps.append((th1 - th0[b]) / e - 0.5 * e * ldg0[b])
            ctx.set_params(b, th0[b].astype(np.float32))   # u = 0 accepts: put the chain back
        return np.array(ps)

    p = draw(1234)
    x = p.ravel()
    N = x.size
    assert abs(x.mean()) < 4.0 / np.sqrt(N), x.mean()
    assert abs(x.var() - 1.0) < 4.0 * np.sqrt(2.0 / N), x.var()
    assert abs(stats.kurtosis(x)) < 4.0 * np.sqrt(24.0 / N)
    assert stats.kstest(x, "norm").pvalue > 1e-3
    assert abs(np.corrcoef(x[:-1], x[1:])[0, 1]) < 4.0 / np.sqrt(N)
    c = np.corrcoef(p)
    assert np.max(np.abs(c[np.triu_indices(nb, 1)])) < 5.0 / np.sqrt(P)
    assert np.allclose(draw(1234), p, atol=1e-3)        # same seed: same momenta (recovery error ~1e-5)
    assert np.max(np.abs(draw(99) - p)) > 1.0           # another seed: other momenta
    ctx.close()


def test_leapfrog_session_matches_hmc_step(Ctx):
    """The benchmark entry points (begin/steps/end, device RNG) run the same
    integrator: with L steps they leave every branch accepted/rejected with
    finite traces and params either moved or restored."""
    rng = np.random.default_rng(21)
    n, M, nb = 512, 640, 5
    g = O.synthetic_genotypes(rng, n, M)
    specs = []
    for b in range(nb):
        snps = np.arange(b * 128, (b + 1) * 128, dtype=np.int32)
        br = f32_branch(O.random_branch(rng, 128, [4, 4, 1]))
        specs.append(dict(snps=snps, branch=br, y=rng.normal(size=n)))
    ctx = build_context(Ctx, g, specs)
    before = [ctx.get_params(b) for b in range(nb)]
    ctx.leapfrog_begin(list(range(nb)), 8, 10.0, "izmailov", 0.5, seed=3)
    ctx.leapfrog_steps(3)
    ctx.leapfrog_steps(5)
    status, acc = ctx.leapfrog_end()
    assert acc == int(np.sum(status == 0))
    for b in range(nb):
        after = ctx.get_params(b)
        assert np.all(np.isfinite(after))
        if status[b] != 0:
            assert np.array_equal(after, before[b])
    ctx.close()


@pytest.mark.parametrize("n", [1003, 2048])
def test_residual_delta_matches_oracle(Ctx, n):
    """residual change of a trajectory (net.rs:279-300 bookkeeping): the sum over
    accepted branches of f_b(theta_L) - f_b(theta_0), from both the host and the
    device entry points, against the oracle predictions of the same params."""
    rng = np.random.default_rng(5 + n)
    nb, m = 37, 64
    g = O.synthetic_genotypes(rng, n, nb * m)
    specs = []
    for b in range(nb):
        br = f32_branch(O.random_branch(rng, m, [4, 4, 1]))
        specs.append(dict(snps=np.arange(b * m, (b + 1) * m, dtype=np.int32), branch=br, y=rng.normal(size=n)))
    ctx = build_context(Ctx, g, specs)
    mu, sd = ctx.genotype_stats()
    before = [ctx.get_params(b) for b in range(nb)]
    ctx.leapfrog_begin(list(range(nb)), 6, 1.0, "izmailov", 0.5, seed=9)
    ctx.leapfrog_steps(6)
    status, acc = ctx.leapfrog_end()
    assert acc > 0
    got = ctx.residual_delta().astype(np.float64)
    ref = np.zeros(n)
    for b in range(nb):
        if status[b] != 0:
            continue
        X = x_std(g[b * m:(b + 1) * m], mu[b * m:(b + 1) * m], sd[b * m:(b + 1) * m])
        br = specs[b]["branch"]
        w1, b1 = layer_views(br, ctx.get_params(b))
        w0, b0 = layer_views(br, before[b])
        new, old = br.copy(), br.copy()
        new.weights, new.biases = w1, b1
        old.weights, old.biases = w0, b0
        ref += O.predict(new, X) - O.predict(old, X)
    assert np.max(np.abs(got - ref)) <= 1e-4 * max(1.0, np.max(np.abs(ref)))
    ctx.close()


# ------------------------------------------------------------ genotype ingestion
def test_bed_decode_gpu(Ctx):
    bs = KAT["bed_small"]
    ctx = Ctx(0)
    ctx.upload_bed(bytes.fromhex(bs["bed_payload_hex"]), bs["n"], bs["m"])
    g = ctx.download_genotypes(np.arange(bs["m"]))
    assert np.array_equal(g.reshape(-1).astype(np.float32), np.array(bs["data_f32_col_major"], np.float32))
    mu, sd = ctx.genotype_stats()
    assert np.allclose(mu, bs["col_means"], rtol=0, atol=1e-6)
    assert np.allclose(sd, bs["col_stds"], rtol=1e-6, atol=1e-7)
    ctx.close()


def test_synthetic_genotypes_gpu(Ctx):
    ctx = Ctx(0)
    n, M = 5000, 300
    ctx.synthetic_genotypes(n, M, seed=42)
    g = ctx.download_genotypes(np.arange(M))
    assert set(np.unique(g)) <= {0, 1, 2}
    mu, sd = ctx.genotype_stats()
    assert np.all(sd > 0)                                   # zero-variance markers redrawn
    assert np.allclose(mu, g.mean(axis=1), atol=1e-6)
    assert np.allclose(sd, g.astype(np.float64).std(axis=1), rtol=1e-5)
    p = mu / 2
    assert p.min() > 0.0 and p.max() < 0.56                 # p_j ~ U(0.01, 0.5)
    ctx2 = Ctx(0)
    ctx2.synthetic_genotypes(n, M, seed=42)
    assert np.array_equal(ctx2.download_genotypes(np.arange(M)), g)   # counter-based: reproducible
    ctx.close()
    ctx2.close()


def test_error_paths(Ctx):
    from bann import BannError
    ctx = Ctx(0)
    with pytest.raises(BannError):
        ctx.finalize()                                      # no genotypes
    ctx.synthetic_genotypes(64, 10)
    with pytest.raises(BannError):
        ctx.add_branch([0, 11], [4, 1])                     # marker out of range
    with pytest.raises(BannError):
        ctx.add_branch([0, 1], [4, 2])                      # output width != 1
    ctx.add_branch([0, 1, 2], [2, 1])
    ctx.finalize()
    with pytest.raises(BannError):
        ctx.add_branch([0], [1, 1])                         # after finalize
    ctx.close()


# ------------------------------------------------ fx kernel specifics
def test_default_fused_kernel_is_fx(Ctx):
    """The product path is the wave-per-tile kernel on 2-bit genotypes."""
    rng, g, snps, br = make_problem(dict(n=300, m=100, widths=[4, 4, 1], act="tanh", prior="ridge_ard"), 5)
    ctx = build_context(Ctx, g, [dict(snps=snps, branch=br, y=rng.normal(size=300))])
    assert ctx.kernel_path(0) == "fused"
    assert ctx.fused_kernel_name() == "k_fused_grad_fx"
    # 2-bit image: ceil(n / 64) tiles x ceil(m / 64) chunks x 1 KiB
    assert ctx.packed_genotype_bytes == ((300 + 63) // 64) * ((100 + 63) // 64) * 1024
    ctx.close()


@pytest.mark.parametrize("growth", [1.0, 300.0, 1e5])
def test_delta_scale_growth(Ctx, growth):
    """delta0 grows along the individuals (later tiles have residuals up to
    `growth` x larger): the kernel's running per-column digit scale must be
    rescaled exactly (shr_digits) -- parity with the oracle at every growth."""
    n, m = 6000, 320
    rng, g, snps, br = make_problem(dict(n=n, m=m, widths=[4, 4, 1], act="tanh", prior="ridge_ard"), 11)
    ctx = build_context(Ctx, g, [dict(snps=snps, branch=br, y=np.zeros(n))])
    X = oracle_inputs(ctx, g, snps)
    f = O.predict(br, X)
    ramp = np.exp(np.linspace(0.0, np.log(growth), n)) if growth > 1 else np.ones(n)
    y = (f + ramp * rng.normal(size=n)).astype(np.float32).astype(np.float64)
    ctx.set_target(0, y)
    grad, rss = ctx.log_density_gradient(0)
    ogw, ogb, orss = O.log_density_gradient(br, X, y)
    gw, gb = layer_views(br, grad)
    for l in range(br.num_layers):
        assert norm_rel(gw[l], ogw[l]) < TOL, ("W", l, norm_rel(gw[l], ogw[l]))
    for l in range(br.num_layers - 1):
        assert norm_rel(gb[l], ogb[l]) < TOL, ("b", l, norm_rel(gb[l], ogb[l]))
    assert scalar_close(rss, orss), (rss, orss)
    ctx.close()


def test_c3_shape_branch_parity(Ctx):
    """One branch of the bench cohort's shape (n = 50 000, m = 500, W = S = 4):
    782 tiles over many work items and all four waves of each."""
    n, m = 50_000, 500
    rng, g, snps, br = make_problem(dict(n=n, m=m, widths=[4, 4, 1], act="tanh", prior="ridge_ard"), 21)
    ctx = build_context(Ctx, g, [dict(snps=snps, branch=br, y=np.zeros(n))])
    X = oracle_inputs(ctx, g, snps)
    f = O.predict(br, X)
    y = (f + rng.normal(scale=max(float(np.std(f)), 0.1), size=n)).astype(np.float32).astype(np.float64)
    ctx.set_target(0, y)
    grad, rss = ctx.log_density_gradient(0)
    ogw, ogb, orss = O.log_density_gradient(br, X, y)
    assert norm_rel(grad, O.param_vec(ogw, ogb)) < TOL
    gw, gb = layer_views(br, grad)
    for l in range(br.num_layers):
        assert norm_rel(gw[l], ogw[l]) < TOL, ("W", l, norm_rel(gw[l], ogw[l]))
    assert scalar_close(rss, orss), (rss, orss)
    assert norm_rel(ctx.predict(0), f) < TOL
    ctx.close()


def test_default_arch_full_n(Ctx):
    """One branch of the reference's default architecture (W = S = m_b / 2,
    cli.rs:365-375) at the bench cohort's n = 50 000: the gx GEMMs over 782 row
    tiles, 13 row splits of the gradient GEMMs and 4 column tiles per layer."""
    n, m = 50_000, 500
    rng, g, snps, br = make_problem(dict(n=n, m=m, widths=[250, 250, 1], act="tanh", prior="ridge_ard"), 23)
    ctx = build_context(Ctx, g, [dict(snps=snps, branch=br, y=np.zeros(n))])
    assert ctx.kernel_path(0) == "layered"
    X = oracle_inputs(ctx, g, snps)
    f = O.predict(br, X)
    y = (f + rng.normal(scale=max(float(np.std(f)), 0.1), size=n)).astype(np.float32).astype(np.float64)
    ctx.set_target(0, y)
    grad, rss = ctx.log_density_gradient(0)
    ogw, ogb, orss = O.log_density_gradient(br, X, y)
    gw, gb = layer_views(br, grad)
    for l in range(br.num_layers):
        assert norm_rel(gw[l], ogw[l]) < TOL, ("W", l, norm_rel(gw[l], ogw[l]))
    for l in range(br.num_layers - 1):
        assert norm_rel(gb[l], ogb[l]) < TOL, ("b", l, norm_rel(gb[l], ogb[l]))
    assert scalar_close(rss, orss), (rss, orss)
    assert norm_rel(ctx.predict(0), f) < TOL
    ctx.close()


@pytest.mark.parametrize("exact", ["0", "1"])
def test_layered_masked_layer_modes(Ctx, exact):
    """gx's GEMMs on the bf16 MFMA (default: the masked layer with the genotype codes
    exact and the f32 operand as three bf16 planes; the hidden layers with both f32
    operands as three planes and the six leading plane products) and on the f32
    MFMA (BANN_GX_EXACT=1): both within the 1e-5 tolerance on a default-architecture
    branch with several row splits."""
    cfg = dict(n=9000, m=300, widths=[150, 150, 1], act="tanh", prior="ridge_ard")
    rng, g, snps, br = make_problem(cfg, 47)
    os.environ["BANN_GX_EXACT"] = exact
    try:
        ctx = build_context(Ctx, g, [dict(snps=snps, branch=br, y=np.zeros(cfg["n"]))])
        X = oracle_inputs(ctx, g, snps)
        f = O.predict(br, X)
        y = (f + rng.normal(scale=max(float(np.std(f)), 0.1), size=cfg["n"])).astype(np.float32).astype(np.float64)
        ctx.set_target(0, y)
        grad, rss = ctx.log_density_gradient(0)
        pred = ctx.predict(0)
    finally:
        del os.environ["BANN_GX_EXACT"]
    from test_oracle_kats import cancellation_tol
    ogw, ogb, orss = O.log_density_gradient(br, X, y)
    gw, gb = layer_views(br, grad)
    for l in range(br.num_layers):
        assert norm_rel(gw[l], ogw[l]) < TOL, ("W", l, norm_rel(gw[l], ogw[l]))
    # bias gradients: sums over 9000 rows of f32 deltas with heavy cancellation; the
    # exact-f32 path lands at 0.5-2e-5 here too (tools/gx_prec.py), so the f32
    # rounding bound of that sum is the tolerance, as for the KAT bias gradients
    for l in range(br.num_layers - 1):
        assert norm_rel(gb[l], ogb[l]) < cancellation_tol(br, X, l, y), ("b", l, norm_rel(gb[l], ogb[l]))
    assert scalar_close(rss, orss) and norm_rel(pred, f) < TOL
    ctx.close()


def test_layered_scratch_groups_and_packing(Ctx):
    """gx branches of mixed shapes in several scratch groups (a 1 MiB budget puts
    every branch in its own group, so later groups overwrite the scratch of
    earlier ones): every gradient matches the oracle, equals the one-group
    result bitwise, and is bitwise reproducible.  The lazy head (kernels_gx.hip:
    delta_s formed while BWD_s / GRAD_s stage A_s) runs for tanh, leaky ReLU and
    identity after one or two hidden layers, beside branches that keep the stored
    head (SiLU, no hidden layer) in the same group."""
    rng = np.random.default_rng(29)
    n, M = 1500, 900
    g = O.synthetic_genotypes(rng, n, M)
    shapes = [(300, [150, 150, 1], "tanh", "ridge_ard"), (70, [35, 1], "relu", "lasso_base"),
              (129, [64, 65, 3, 1], "silu", "ridge_base"), (500, [5, 250, 1], "tanh", "lasso_ard"),
              (180, [90, 60, 30, 1], "tanh", "ridge_ard"), (150, [75, 40, 1], "leaky_relu", "ridge_base"),
              (100, [50, 130, 1], "identity", "lasso_ard")]
    specs = []
    for m, w, a, p in shapes:
        snps = rng.choice(M, size=m, replace=False).astype(np.int32)
        br = f32_branch(O.random_branch(rng, m, w, prior=p, act=a))
        specs.append(dict(snps=snps, branch=br, y=rng.normal(size=n).astype(np.float32).astype(np.float64)))
    grads = []
    for budget in ("1", None):
        if budget:
            os.environ["BANN_GX_SCRATCH_MB"] = budget
        try:
            ctx = build_context(Ctx, g, specs)
        finally:
            os.environ.pop("BANN_GX_SCRATCH_MB", None)
        assert all(ctx.kernel_path(b) == "layered" for b in range(len(specs)))
        mu, sd = ctx.genotype_stats()
        res = ctx.predict_many(list(range(len(specs))))
        gb = []
        for b, s in enumerate(specs):
            X = x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]])
            grad, rss = ctx.log_density_gradient(b)
            ogw, ogb, orss = O.log_density_gradient(s["branch"], X, s["y"])
            assert norm_rel(grad, O.param_vec(ogw, ogb)) < TOL, b
            assert scalar_close(rss, orss)
            assert norm_rel(res[b], O.predict(s["branch"], X)) < TOL
            g2, _ = ctx.log_density_gradient(b)
            assert np.array_equal(grad, g2)
            gb.append(grad)
        grads.append(gb)
        ctx.close()
    for a, b in zip(*grads):
        assert np.array_equal(a, b)


# ------------------------------------------------------------- wide kernel (wx)
def _wide_problem(Ctx, seed, n=2000, m=125, widths=(32, 32, 1), nb=3, act="tanh"):
    rng = np.random.default_rng(seed)
    g = O.synthetic_genotypes(rng, n, nb * m)
    specs = [dict(snps=np.arange(b * m, (b + 1) * m, dtype=np.int32),
                  branch=f32_branch(O.random_branch(rng, m, list(widths), act=act)), y=None) for b in range(nb)]
    ctx = build_context(Ctx, g, [dict(s, y=np.zeros(n)) for s in specs])
    mu, sd = ctx.genotype_stats()
    for b, s in enumerate(specs):
        s["X"] = x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]])
        f = O.predict(s["branch"], s["X"])
        s["y"] = (f + rng.normal(scale=max(float(np.std(f)), 0.1), size=n)).astype(np.float32).astype(np.float64)
        ctx.set_target(b, s["y"])
    return ctx, specs


def test_wide_packed_deterministic(Ctx):
    """C5-shaped branches (m = 125, W = S = 32) packed in one launch: per-branch
    parity, bitwise-reproducible fixed-order reductions, split invariance."""
    ctx, specs = _wide_problem(Ctx, 41)
    assert all(ctx.kernel_path(b) == "wide" for b in range(len(specs)))
    for b, s in enumerate(specs):
        grad, rss = ctx.log_density_gradient(b)
        ogw, ogb, orss = O.log_density_gradient(s["branch"], s["X"], s["y"])
        assert norm_rel(grad, O.param_vec(ogw, ogb)) < TOL, b
        assert scalar_close(rss, orss)
        g2, r2 = ctx.log_density_gradient(b)
        assert np.array_equal(grad, g2) and rss == r2
    many = ctx.predict_many([2, 0, 1])
    for i, b in enumerate([2, 0, 1]):
        assert norm_rel(many[i], O.predict(specs[b]["branch"], specs[b]["X"])) < TOL
    g_ref = ctx.log_density_gradient(1)[0]
    ctx.close()
    os.environ["BANN_TARGET_ITEMS"] = "1"
    try:
        ctx, _ = _wide_problem(Ctx, 41)
        g1 = ctx.log_density_gradient(1)[0]
    finally:
        del os.environ["BANN_TARGET_ITEMS"]
    assert norm_rel(g1, g_ref) < 1e-6
    ctx.close()


def test_wide_exact_f32_path(Ctx):
    """BANN_WX_EXACT=1 keeps the hidden GEMMs on the exact f32 MFMA
    (k_fused_grad_wx, one tile per two-wave workgroup); the default plane path
    (k_fused_grad_wx3: three bf16 planes per f32 operand, six products) and it
    both match the oracle to 1e-5 and each other to f32 rounding."""
    ctx, specs = _wide_problem(Ctx, 45, nb=2, widths=(32, 27, 1))
    g_planes = [ctx.log_density_gradient(b) for b in range(2)]
    ctx.close()
    os.environ["BANN_WX_EXACT"] = "1"
    try:
        ctx, _ = _wide_problem(Ctx, 45, nb=2, widths=(32, 27, 1))
        g_exact = [ctx.log_density_gradient(b) for b in range(2)]
        ctx.close()
    finally:
        del os.environ["BANN_WX_EXACT"]
    for b, s in enumerate(specs):
        ogw, ogb, orss = O.log_density_gradient(s["branch"], s["X"], s["y"])
        ref = O.param_vec(ogw, ogb)
        for grad, rss in (g_planes[b], g_exact[b]):
            assert norm_rel(grad, ref) < TOL, b
            assert scalar_close(rss, orss)
        assert norm_rel(g_planes[b][0], g_exact[b][0]) < 2e-6


def test_wide_bf16_hidden_gemm(Ctx):
    """bann_set_hidden_gemm_bf16 (C5's bf16 hidden GEMM): the hidden-layer GEMMs
    round their operands to bf16 (8-bit mantissa), so the gradient agrees with
    the f32 oracle to ~1e-2 (norm-relative), not 1e-5; the masked layer stays
    exact.  The f32 mode of the same context is parity-exact again."""
    ctx, specs = _wide_problem(Ctx, 43, nb=2)
    ctx.set_hidden_gemm_bf16(True)
    s = specs[0]
    grad, rss = ctx.log_density_gradient(0)
    ogw, ogb, orss = O.log_density_gradient(s["branch"], s["X"], s["y"])
    err = norm_rel(grad, O.param_vec(ogw, ogb))
    assert 0 < err < 3e-2, err
    assert scalar_close(rss, orss, 1e-2)
    ctx.set_hidden_gemm_bf16(False)
    grad, rss = ctx.log_density_gradient(0)
    assert norm_rel(grad, O.param_vec(ogw, ogb)) < TOL
    ctx.close()


def test_c5_shape_wide_full_n(Ctx):
    """BASELINE config C5's branch at its full cohort size (m = 125, W = S = 32,
    n = 100 000): the wide kernel's f32 gradient, rss and prediction match the
    oracle to 1e-5 (dW0 digit sums and the f32 MFMA hidden GEMMs accumulate over
    1 563 tiles); the bf16 hidden-GEMM mode stays within its 3e-2 bound."""
    ctx, specs = _wide_problem(Ctx, 47, n=100_000, nb=2)
    assert all(ctx.kernel_path(b) == "wide" for b in range(2))
    for b, s in enumerate(specs):
        grad, rss = ctx.log_density_gradient(b)
        ogw, ogb, orss = O.log_density_gradient(s["branch"], s["X"], s["y"])
        assert norm_rel(grad, O.param_vec(ogw, ogb)) < TOL, (b, norm_rel(grad, O.param_vec(ogw, ogb)))
        assert scalar_close(rss, orss), (rss, orss)
        assert norm_rel(ctx.predict(b), O.predict(s["branch"], s["X"])) < TOL
    ctx.set_hidden_gemm_bf16(True)
    s = specs[1]
    grad, rss = ctx.log_density_gradient(1)
    ogw, ogb, orss = O.log_density_gradient(s["branch"], s["X"], s["y"])
    assert norm_rel(grad, O.param_vec(ogw, ogb)) < 3e-2
    assert scalar_close(rss, orss, 1e-2)
    ctx.close()


# ------------------------------------------------------------ joint HMC parity
HYPER = (0.5, 2.0, 0.8, 3.0, 1.1, 5.0)   # dense, summary, output (shape, scale)


@pytest.mark.parametrize("shape", [("fx", 60, [4, 4, 1]), ("wide", 40, [8, 8, 1]), ("layered", 30, [6, 5, 3, 1])])
@pytest.mark.parametrize("prior", ["ridge_ard", "ridge_base", "lasso_ard", "lasso_base"])
def test_hmc_step_joint_parity(Ctx, prior, shape):
    """hmc_step_joint (branch_sampler.rs:1070-1178) with injected step sizes,
    momenta and uniform: the joint -H trace (parameter and precision gradients,
    joint log density incl. the other branches' output-weight stat), the status
    (final test on the NON-joint density, the reference quirk), the final
    parameters and the sampled precisions match the oracle."""
    path, m, widths = shape
    rng = np.random.default_rng(31)
    n, L = 500, 6
    g = O.synthetic_genotypes(rng, n, m)
    br = f32_branch(O.random_branch(rng, m, widths, prior=prior, act="tanh"))
    br.out_reg_sum, br.out_num_params = float(np.float32(0.37)), 24.0
    ctx = build_context(Ctx, g, [dict(snps=np.arange(m, dtype=np.int32), branch=br, y=np.zeros(n))])
    assert ctx.kernel_path(0) == {"fx": "fused", "wide": "wide", "layered": "layered"}[path]
    ctx.set_output_stats(0, br.out_reg_sum, br.out_num_params)
    X = oracle_inputs(ctx, g, np.arange(m))
    y = (O.predict(br, X) + rng.normal(scale=0.5, size=n)).astype(np.float32).astype(np.float64)
    ctx.set_target(0, y)
    P, Q = br.num_params, O.precision_vec(br).size
    hp = O.Hyper(dense=HYPER[0:2], summary=HYPER[2:4], output=HYPER[4:6])
    ctx.set_trajectory_recording(True)   # the joint Trajectory (branch_sampler.rs:1126-1135)
    for u, scale in [(0.3, 2e-4), (0.3, 3e-3), (0.5, 1.0)]:   # small, larger, absurd (early rejection)
        eps = (scale * rng.uniform(size=P + Q)).astype(np.float32)
        p0 = rng.normal(size=P + Q).astype(np.float32)
        theta0 = ctx.get_params(0)
        res = ctx.hmc_step_joint([0], L, HYPER, eps=eps, momentum=p0, u=[u])
        ob = br.copy()
        out = O.hmc_step_joint(ob, X, y, hp, eps.astype(np.float64), p0.astype(np.float64), L, 10.0, u)
        assert res["status"][0] == out["status"], (scale, res["status"], out["status"])
        tr = np.asarray(out["trace"])
        gt = res["trace"][0][: tr.size]
        # a diverged step's -H (|dH| ~ 1e10 at scale 1) is f32 noise vs float64: check the status only there
        fin = np.isfinite(tr) & (np.abs(tr - tr[0]) <= 10.0)
        assert np.all(np.abs(gt[fin] - tr[fin]) <= 1e-5 * np.maximum(1.0, np.abs(tr[fin]))), (scale, gt, tr)
        rec = ctx.get_trajectory_joint(0)
        k = len(out["states"])
        assert rec["params"].shape == (k, P) and rec["precisions"].shape == (k, Q) and rec["ldg"].shape == (k, P + Q)
        assert np.array_equal(rec["hamiltonian"], res["trace"][0][: k + 1])
        for j in range(k):
            if fin[j + 1]:
                assert norm_rel(rec["params"][j], out["states"][j][:P]) < 1e-5, (scale, j)
                assert norm_rel(rec["precisions"][j], out["states"][j][P:]) < 1e-5, (scale, j)
                assert norm_rel(rec["ldg"][j], out["ldgs"][j]) < 1e-5, (scale, j)
        with pytest.raises(Exception):   # the parameter-only getter refuses a joint recording
            ctx.get_trajectory(0)
        assert norm_rel(ctx.get_params(0), O.param_vec(ob.weights, ob.biases)) < 1e-5
        assert norm_rel(ctx.get_precisions(0), O.precision_vec(ob)) < 1e-5
        if out["status"] != O.REJECTED_EARLY:
            assert scalar_close(res["log_density"][0], out["log_density"]), (res["log_density"], out["log_density"])
        if out["status"] != O.ACCEPTED:
            assert np.array_equal(ctx.get_params(0), theta0)
        br = ob
    ctx.close()


@pytest.mark.parametrize("shape", [("fx", 60, [4, 4, 1]), ("fxl", 700, [4, 3, 1]), ("wide", 40, [8, 8, 1]),
                                   ("layered", 30, [6, 5, 3, 1]), ("layered", 90, [45, 45, 1])])
@pytest.mark.parametrize("act", ["tanh", "relu", "silu"])
def test_forward_feed_every_layer(Ctx, shape, act):
    """bann_forward_feed (forward_feed, branch_sampler.rs:743-782, every layer
    kept, for Net::activations net.rs:509-518): the pre-activations and
    activations of every layer match the oracle on every kernel path's shapes."""
    path, m, widths = shape
    rng = np.random.default_rng(7)
    n = 333
    g = O.synthetic_genotypes(rng, n, m)
    br = f32_branch(O.random_branch(rng, m, widths, act=act))
    ctx = build_context(Ctx, g, [dict(snps=np.arange(m, dtype=np.int32), branch=br, y=np.zeros(n))])
    X = oracle_inputs(ctx, g, np.arange(m))
    pre, act_ = ctx.forward_feed(0)
    opre, oact = O.forward_feed(br, X)
    assert len(pre) == len(opre) == len(widths) - 1 and len(act_) == len(oact) == len(widths)
    for a, oa in zip(pre + act_, opre + oact):
        assert a.shape == oa.shape and norm_rel(a, oa) < 1e-5
    ctx.close()


def test_gradient_many_and_joint_gradient(Ctx):
    """bann_log_density_gradient_many (one packed launch, Net::gradient) equals
    the per-branch calls bitwise; bann_log_density_gradient_joint
    (log_density_gradient_joint, branch_sampler.rs:406-422) and its joint log
    density (292-305) match the oracle for ridge / lasso, ARD / base."""
    rng = np.random.default_rng(19)
    n = 640
    shapes = [(60, [4, 4, 1], "ridge_ard"), (40, [8, 8, 1], "lasso_base"), (30, [6, 5, 3, 1], "lasso_ard"),
              (700, [4, 3, 1], "ridge_base")]
    g = O.synthetic_genotypes(rng, n, sum(m for m, _, _ in shapes))
    specs, off = [], 0
    for m, w, prior in shapes:
        br = f32_branch(O.random_branch(rng, m, w, prior=prior))
        br.out_reg_sum, br.out_num_params = float(np.float32(0.21)), 17.0
        specs.append(dict(snps=np.arange(off, off + m, dtype=np.int32), branch=br,
                          y=rng.normal(size=n).astype(np.float32)))
        off += m
    ctx = build_context(Ctx, g, specs)
    grads, rss = ctx.log_density_gradient_many([3, 0, 2, 1])
    for gv, r, b in zip(grads, rss, [3, 0, 2, 1]):
        g1, r1 = ctx.log_density_gradient(b)
        assert np.array_equal(gv, g1) and r == r1, b
    hp = O.Hyper(dense=HYPER[0:2], summary=HYPER[2:4], output=HYPER[4:6])
    for b, s in enumerate(specs):
        br = s["branch"]
        ctx.set_output_stats(b, br.out_reg_sum, br.out_num_params)
        X = oracle_inputs(ctx, g, s["snps"])
        yd = s["y"].astype(np.float64)
        gj, r, ld = ctx.log_density_gradient_joint(b, HYPER)
        og, orss = O.ldg_joint_vec(br, X, yd, hp)
        P = br.num_params
        assert norm_rel(gj[:P], og[:P]) < 1e-5 and norm_rel(gj[P:], og[P:]) < 1e-5, b
        assert scalar_close(r, orss), b
        old = O.log_density_joint(br, orss, hp, n)
        assert scalar_close(ld, old), (b, ld, old)
    ctx.close()


def test_graph_replay_matches_launches(Ctx):
    """bann_set_graph_replay: a trajectory replayed as one captured HIP graph
    gives the bits of the launch-by-launch trajectory -- status, -H trace,
    parameters and prediction rows -- over several branch sets and L (graphs are
    keyed by plan shape, L and the kernels' by-value state; fxl branches of 4 and
    8 marker chunks per wave -- different templates and LDS sizes -- included)."""
    rng = np.random.default_rng(41)
    n = 900
    shapes = [(60, [4, 4, 1]), (120, [4, 3, 1]), (40, [8, 8, 1]), (30, [6, 5, 3, 1]), (1300, [4, 4, 1]),
              (2200, [4, 4, 1])]
    g = O.synthetic_genotypes(rng, n, sum(m for m, _ in shapes))
    specs, off = [], 0
    for m, w in shapes:
        br = f32_branch(O.random_branch(rng, m, w))
        specs.append(dict(snps=np.arange(off, off + m, dtype=np.int32), branch=br,
                          y=rng.normal(size=n).astype(np.float32)))
        off += m
    ctxs = [build_context(Ctx, g, specs) for _ in range(2)]
    ctxs[1].set_graph_replay(True)
    assert ctxs[0].kernel_path(4) == ctxs[0].kernel_path(5) == "fused_large"
    for it, (bl, L) in enumerate([([0], 3), ([0, 1], 5), ([2], 4), ([0], 3), ([3, 1], 6), ([0, 1], 5), ([4], 3),
                                  ([5], 3), ([4, 5], 4), ([4], 3), ([5], 3)]):
        out = [c.hmc_step(bl, L, 10.0, step_factor=0.3, seed=100 + it) for c in ctxs]
        assert np.array_equal(out[0]["status"], out[1]["status"]), it
        assert np.array_equal(out[0]["trace"], out[1]["trace"], equal_nan=True), it
        for b in range(len(shapes)):
            assert np.array_equal(ctxs[0].get_params(b), ctxs[1].get_params(b)), (it, b)
            assert np.array_equal(ctxs[0].predict(b), ctxs[1].predict(b)), (it, b)
    for c in ctxs:
        c.close()


def test_hmc_step_joint_refuses_std_normal_and_reports_shapes(Ctx):
    rng = np.random.default_rng(3)
    n, m = 100, 20
    g = O.synthetic_genotypes(rng, n, m)
    br = f32_branch(O.random_branch(rng, m, [4, 1], prior="std_normal"))
    ctx = build_context(Ctx, g, [dict(snps=np.arange(m), branch=br, y=np.zeros(n))])
    from bann import BannError
    with pytest.raises(BannError):
        ctx.hmc_step_joint([0], 3, HYPER)
    with pytest.raises(ValueError):   # eps must cover parameters AND precisions
        ctx.hmc_step_joint([0], 3, HYPER, eps=np.ones(br.num_params, np.float32))
    ctx.close()


# ------------------------------------------------------------ ingestion (f3)
PLINK = os.path.join(HERE, "golden", "plink")


def test_load_bed_file_small_and_random(Ctx):
    """bann_genotypes_load_bed streams stem.bed into the 2-bit device image: the
    reference's small fileset (dims from .fam/.bim) decodes to the matrix of
    resources/test/README.md with the reference's column statistics; random.bed
    (dims from random.dims) decodes like the oracle's bed_decode of its bytes."""
    bs = KAT["bed_small"]
    ctx = Ctx(0)
    ctx.load_bed(os.path.join(PLINK, "small"))
    g = ctx.download_genotypes(np.arange(bs["m"]))
    assert np.array_equal(g.reshape(-1).astype(np.float32), np.array(bs["data_f32_col_major"], np.float32))
    mu, sd = ctx.genotype_stats()
    assert np.allclose(mu, bs["col_means"], rtol=0, atol=1e-6)
    assert np.allclose(sd, bs["col_stds"], rtol=1e-6, atol=1e-7)
    ctx.close()
    raw = open(os.path.join(PLINK, "random.bed"), "rb").read()
    ctx = Ctx(0)
    ctx.load_bed(os.path.join(PLINK, "random"))
    g = ctx.download_genotypes(np.arange(20))
    assert np.array_equal(g, O.bed_decode(raw[3:], 100, 20))
    ctx.close()


def test_upload_paths_agree_and_reject_non_2bit(Ctx):
    """int8 upload (streamed, packed on the device), .bed payload upload and
    download agree bit for bit; an int8 value outside 0..3 is refused."""
    rng = np.random.default_rng(12)
    n, M = 1003, 77
    g = O.synthetic_genotypes(rng, n, M)
    a = Ctx(0)
    a.upload_genotypes(g)
    b = Ctx(0)
    b.upload_bed(O.bed_encode(g), n, M)
    assert np.array_equal(a.download_genotypes(np.arange(M)), g)
    assert np.array_equal(b.download_genotypes(np.arange(M)), g)
    for x, y in zip(a.genotype_stats(), b.genotype_stats()):
        assert np.array_equal(x, y)
    a.close()
    b.close()
    from bann import BannError
    bad = g.copy()
    bad[3, 5] = 4
    c = Ctx(0)
    with pytest.raises(BannError):
        c.upload_genotypes(bad)
    c.close()


@pytest.mark.parametrize("n", [1000, 4093])
def test_forward_fi_matches_lds_forward(Ctx, n, monkeypatch):
    """the forward-only pass over the individual-major fi images
    (kernels_fi.hip: plain global loads into the i8 MFMA, the group's tiles cut
    into equal per-wave ranges across branch boundaries) gives the bits of the
    LDS forward (k_forward_fx, BANN_FWD_FI=0) for every fx shape -- one and two
    256-marker segments, 2 to 4 layers, every activation -- and the oracle's
    predictions (forward_feed, branch_sampler.rs:743-782)."""
    rng = np.random.default_rng(n)
    shapes = [(60, [4, 4, 1], "tanh"), (256, [4, 1], "relu"), (300, [3, 4, 1], "silu"), (512, [4, 4, 4, 1], "tanh"),
              (17, [2, 3, 1], "leaky_relu"), (500, [4, 4, 1], "identity"), (129, [4, 4, 1], "tanh")]
    g = O.synthetic_genotypes(rng, n, sum(m for m, _, _ in shapes))
    specs, off = [], 0
    for m, w, act in shapes:
        specs.append(dict(snps=np.arange(off, off + m, dtype=np.int32),
                          branch=f32_branch(O.random_branch(rng, m, w, act=act)), y=np.zeros(n)))
        off += m
    preds = []
    for fi in ("0", "1"):
        monkeypatch.setenv("BANN_FWD_FI", fi)
        ctx = build_context(Ctx, g, specs)
        assert all(ctx.kernel_path(b) == "fused" for b in range(len(specs)))
        preds.append(ctx.predict_many(list(range(len(specs)))))
        if fi == "1":
            sub = ctx.predict_many([5, 1, 3])   # another plan: other items, other cut points
            assert np.array_equal(sub, preds[1][[5, 1, 3]])
            mu, sd = ctx.genotype_stats()
            for b, s in enumerate(specs):
                X = x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]])
                assert norm_rel(preds[1][b], O.predict(s["branch"], X)) < 1e-5, b
        ctx.close()
    assert np.array_equal(preds[0], preds[1])


@pytest.mark.parametrize("shape,fused", [("multi", "1"), ("single", "1")])
def test_fused_update_session_bitwise(Ctx, monkeypatch, shape, fused):
    """the leapfrog update in the gradient launch's tail (update_small as 512
    virtual threads) gives the bits of the separate update launches
    (BANN_FUSE_UPDATE=0): statuses, parameters, predictions.
      multi: a one-round multi-split fx plan (the N = 8 shard's shape: here 70
        branches x 7 splits), the last arriving workgroup of each branch updates
        it (BANN_FUSE_UPDATE=1);
      single: one split per branch (C3's shape: 600 branches on 1 024
        individuals), each branch's one workgroup updates it (BANN_FUSE_UPDATE=1)."""
    rng = np.random.default_rng(77)
    n, nb, m = (2048, 70, 60) if shape == "multi" else (1024, 600, 20)
    g = O.synthetic_genotypes(rng, n, nb * m)
    specs = []
    for b in range(nb):
        specs.append(dict(snps=np.arange(b * m, (b + 1) * m, dtype=np.int32),
                          branch=f32_branch(O.random_branch(rng, m, [4, 4, 1])),
                          y=rng.normal(size=n).astype(np.float32)))
    outs = []
    for fuse in ("0", fused):
        if fuse is None:
            monkeypatch.delenv("BANN_FUSE_UPDATE", raising=False)
        else:
            monkeypatch.setenv("BANN_FUSE_UPDATE", fuse)
        ctx = build_context(Ctx, g, specs)   # single: 600 branches -> 1 split each (bann_api.hip best_splits)
        res = []
        for traj, (L, f) in enumerate([(5, 0.05), (3, 2.0), (8, 0.02)]):
            ctx.leapfrog_begin(list(range(nb)), L, 10.0, "izmailov", f, seed=3 + traj)
            ctx.leapfrog_steps(L)
            st, acc = ctx.leapfrog_end()
            res.append((st.copy(), acc, [ctx.get_params(b) for b in range(nb)], ctx.residual_delta()))
        outs.append(res)
        ctx.close()
    for (s0, a0, p0, d0), (s1, a1, p1, d1) in zip(*outs):
        assert np.array_equal(s0, s1) and a0 == a1
        for b in range(nb):
            assert np.array_equal(p0[b], p1[b]), b
        assert np.array_equal(d0, d1)
    assert sum(a for _, a, _, _ in outs[1]) > 0   # some trajectory accepted: the fused tail moved the chain


@pytest.mark.parametrize("graph", [False, True])
def test_fused_solo_hmc_step_bitwise(Ctx, monkeypatch, graph):
    """the sequential driver's single-branch trajectories (solo plans: the branch
    re-split over many workgroups): with the fold and the update in the gradient
    launch's tail (BANN_FUSE_UPDATE=1: the last arriving workgroup adds the branch's
    slabs in k_fold_solo's order, then updates it) every trajectory -- status, -H
    trace, parameters, prediction rows -- has the bits of the separate fold and
    update launches (the default), launched one by one or replayed as a graph."""
    rng = np.random.default_rng(83)
    n, nb, m = 20000, 3, 500
    g = O.synthetic_genotypes(rng, n, nb * m)
    specs = [dict(snps=np.arange(b * m, (b + 1) * m, dtype=np.int32),
                  branch=f32_branch(O.random_branch(rng, m, [4, 4, 1])),
                  y=rng.normal(size=n).astype(np.float32)) for b in range(nb)]
    monkeypatch.setenv("BANN_SOLO_TPW", "4")   # the same solo split in both contexts
    outs = []
    for fuse in ("0", "1"):
        monkeypatch.setenv("BANN_FUSE_UPDATE", fuse)
        ctx = build_context(Ctx, g, specs)
        ctx.set_graph_replay(graph)
        res = []
        for it, (b, L, f) in enumerate([(0, 5, 0.3), (1, 3, 1.0), (2, 6, 0.2), (0, 4, 0.5), (1, 5, 0.05)]):
            r = ctx.hmc_step([b], L, 10.0, step_factor=f, seed=500 + it)
            res.append((r["status"].copy(), r["trace"].copy(), [ctx.get_params(k) for k in range(nb)],
                        [ctx.predict(k) for k in range(nb)]))
        outs.append(res)
        ctx.close()
    acc = 0
    for (s0, t0, p0, f0), (s1, t1, p1, f1) in zip(*outs):
        assert np.array_equal(s0, s1)
        assert np.array_equal(t0, t1, equal_nan=True)
        for k in range(nb):
            assert np.array_equal(p0[k], p1[k]), k
            assert np.array_equal(f0[k], f1[k]), k
        acc += int(s1[0] == 0)
    assert acc > 0


def test_fxh_head_wave_kernel(Ctx):
    """k_fused_grad_fxh (fxl shapes of 17..32 chunks: one head wave, compute waves
    of <= 5 chunks, two-tile software pipeline): oracle gradients, rss and
    predictions for ragged chunk partitions (18, 21, 27 and 32 chunks over 4..7
    compute waves; 2, 3 and 4 layers), in solo plans (one or two tiles per item:
    the pipeline's prologue / epilogue) and in long items (BANN_SOLO=0), packed
    and one branch at a time; and fxl (BANN_FXL_HEAD=0) agrees to f32 rounding."""
    rng = np.random.default_rng(41)
    n = 3000
    shapes = [(1100, [4, 4, 1], "tanh"), (1300, [3, 2, 1], "relu"), (1700, [4, 4, 4, 1], "silu"),
              (2048, [4, 1], "tanh")]
    M = sum(m for m, _, _ in shapes)
    g = O.synthetic_genotypes(rng, n, M)
    specs, off = [], 0
    for m, w, a in shapes:
        br = f32_branch(O.random_branch(rng, m, w, act=a))
        specs.append(dict(snps=np.arange(off, off + m, dtype=np.int32), branch=br,
                          y=rng.normal(size=n).astype(np.float32).astype(np.float64)))
        off += m
    res = {}
    mu = sd = None
    for mode, solo in (("1", None), ("1", "0"), ("0", "0")):
        os.environ["BANN_FXL_HEAD"] = mode
        if solo is not None:
            os.environ["BANN_SOLO"] = solo
        try:
            ctx = build_context(Ctx, g, specs)
            assert all(ctx.kernel_path(b) == "fused_large" for b in range(len(specs)))
            mu, sd = ctx.genotype_stats()
            many, rss_many = ctx.log_density_gradient_many(list(range(len(specs))))
            single = [ctx.log_density_gradient(b) for b in range(len(specs))]
            preds = [ctx.predict(b) for b in range(len(specs))]
            again, _ = ctx.log_density_gradient_many(list(range(len(specs))))
            ctx.close()
        finally:
            del os.environ["BANN_FXL_HEAD"]
            os.environ.pop("BANN_SOLO", None)
        for a, b_ in zip(many, again):
            assert np.array_equal(a, b_)  # fixed-order reductions: bitwise reproducible
        res[(mode, solo)] = (many, rss_many, single, preds)
    for key, (many, rss_many, single, preds) in res.items():
        for b, s in enumerate(specs):
            X = x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]])
            ogw, ogb, orss = O.log_density_gradient(s["branch"], X, s["y"])
            ref = O.param_vec(ogw, ogb)
            assert norm_rel(many[b], ref) < TOL, (key, b, norm_rel(many[b], ref))
            assert norm_rel(single[b][0], ref) < TOL, (key, b)
            assert scalar_close(rss_many[b], orss) and scalar_close(single[b][1], orss), (key, b)
            assert norm_rel(preds[b], O.predict(s["branch"], X)) < TOL, (key, b)
    for b in range(len(specs)):
        assert norm_rel(res[("1", "0")][0][b], res[("0", "0")][0][b]) < 1e-6, b
