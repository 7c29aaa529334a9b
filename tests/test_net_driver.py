"""GPU parity of the sequential network driver (include/bann_net.h: Net::train,
net.rs:201-358, and the Net<B> model file, net.rs:107-115) against the CPU
oracle (oracle/net_oracle.py).

The device driver's RNG hooks replay the same numpy stream the oracle draws
from (draw order: include/bann_net.h), so both take the same Gibbs draws,
momenta, acceptance uniforms and branch orders.  The device computes in f32
(int8 genotypes, exact integer MFMA on the fused path), the oracle in f64; over
a chain of 3 sweeps x 3 branches x 10 leapfrog steps the per-step differences
(<= 1e-5, test_gpu_parity.py) feed back through the residual and the Gibbs
draws, so the chain-level tolerance is 1e-4 (norm-relative for parameter
vectors, relative for scalars).
"""
import json
import os

import numpy as np
import pytest

import bann_oracle as O
import net_oracle as NO
from helpers import f32_branch, norm_rel, x_std

pytestmark = pytest.mark.gpu
CHAIN_TOL = 1e-4


def build(prior, seed=3, n=700, ms=(40, 64, 30), widths=((4, 4, 1), (4, 4, 1), (5, 3, 1))):
    from bann import BannContext
    rng = np.random.default_rng(seed)
    g = O.synthetic_genotypes(rng, n, sum(ms))
    ctx = BannContext(0)
    ctx.upload_genotypes(g)
    branches, snps, off = [], [], 0
    for m, w in zip(ms, widths):
        s = np.arange(off, off + m, dtype=np.int32)
        off += m
        branches.append(f32_branch(O.random_branch(rng, m, list(w), prior=prior)))
        snps.append(s)
        ctx.add_branch(s, list(w), "tanh", prior)
    ctx.finalize()
    op = branches[0].weight_precisions[-1].copy()   # one output-layer precision (architectures.rs:215)
    for b, br in enumerate(branches):
        br.weight_precisions[-1] = op.copy()
        ctx.set_params(b, O.param_vec(br.weights, br.biases))
        ctx.set_precisions(b, O.precision_vec(br))
    mu, sd = ctx.genotype_stats()
    X = [x_std(g[s], mu[s], sd[s]) for s in snps]
    truth = [O.random_branch(rng, m, list(w), prior=prior) for m, w in zip(ms, widths)]
    f = sum(O.predict(t, x) for t, x in zip(truth, X))
    y = (f + rng.normal(scale=0.5 * float(np.std(f)) + 1e-3, size=n)).astype(np.float32)
    return ctx, branches, X, y


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-12)


@pytest.mark.parametrize("prior,opts", [
    ("ridge_ard", {}), ("ridge_ard", dict(sampled_output_bias=True)), ("lasso_base", {}),
    ("lasso_ard", dict(sampled_output_bias=True)),
    # MCMCCfg::joint_hmc: hmc_step_joint, no Gibbs draws (net.rs:270-290)
    ("ridge_ard", dict(joint_hmc=True, factor=0.5)), ("lasso_base", dict(joint_hmc=True, factor=0.5)),
    # StepSizeMode::Random (branch_sampler.rs:654-681, 1212-1217)
    ("ridge_base", dict(step_mode="random")),
    # StepSizeMode::StdScaled (ridge_base.rs:52-82, lasso_base.rs:53-82, dispatched at 1213)
    ("ridge_base", dict(step_mode="std_scaled", factor=0.05)),
    ("lasso_base", dict(step_mode="std_scaled", factor=0.05, sampled_output_bias=True)),
    # Net::train_single_branch (net.rs:360-507)
    ("ridge_ard", dict(single_branch=True)),
    # MCMCCfg::gradient_descent (line search over rss probes, branch_sampler.rs:964-1016)
    ("ridge_ard", dict(gradient_descent=True, factor=1e-4)), ("lasso_ard", dict(gradient_descent=True, factor=1e-4)),
    # MCMCCfg::gradient_descent_joint (params and precisions, 1019-1066)
    ("ridge_ard", dict(gradient_descent_joint=True, factor=1e-5)),
    ("lasso_base", dict(gradient_descent_joint=True, factor=1e-5)),
])
def test_train_matches_oracle(prior, opts):
    from bann import MCMCConfig, Net
    ctx, branches, X, y = build(prior)
    hp = O.Hyper()
    net = Net(ctx, (hp.dense, hp.summary, hp.output))
    d_dev, d_ora = NO.Draws(11), NO.Draws(11)
    net.set_rng(d_dev.uniform, d_dev.normal, d_dev.gamma)
    sampled_bias = opts.get("sampled_output_bias", False)
    factor = opts.get("factor", 1.0)
    single = opts.get("single_branch", False)
    gd, gdj = opts.get("gradient_descent", False), opts.get("gradient_descent_joint", False)
    cfg = MCMCConfig(hmc_integration_length=10, chain_length=3, sampled_output_bias=sampled_bias,
                     hmc_step_size_factor=factor, hmc_step_size_mode=opts.get("step_mode", "izmailov"),
                     joint_hmc=opts.get("joint_hmc", False), gradient_descent=gd, gradient_descent_joint=gdj)
    (net.train_single_branch if single else net.train)(y, cfg)
    ora = NO.NetOracle(branches, X, hp)
    ora.train(y.astype(np.float64), d_ora, 3, 10, factor=factor, step_mode=opts.get("step_mode", "izmailov"),
              sampled_output_bias=sampled_bias, joint_hmc=opts.get("joint_hmc", False), single_branch=single,
              gradient_descent=gd, gradient_descent_joint=gdj)
    assert d_dev.uniform() == d_ora.uniform(), "draw streams diverged (different number of draws)"
    s = net.summary()
    assert (s["num_samples"], s["num_accepted"], s["num_early_rejected"]) == (ora.ns, ora.nacc, ora.nearly)
    mse, lpd = net.records()
    assert len(mse) == len(ora.mse) == 4
    for a, b in zip(mse, ora.mse):
        assert rel(a, b) < CHAIN_TOL, (mse, ora.mse)
    for a, b in zip(lpd, ora.lpd):
        assert rel(a, b) < CHAIN_TOL, (lpd, ora.lpd)
    # gradient descent: where the ascent direction raises the rss, the halving line
    # search (branch_sampler.rs:983-989) runs until a halved step stops lowering the
    # rss -- in f32 (device and reference) where the probe's change sinks below the
    # rounding of the rss (steps ~1e-9), in the float64 oracle at ~1e-17 (measured
    # step by step: tools/diag/gd_trace.py).  Both stopping steps move theta by
    # < 1e-8 relative, but the chain feeds the difference back through the Gibbs
    # draws: 6e-4 after 3 sweeps of lasso_ard, hence 1e-3 for the parameters there.
    ptol = 1e-3 if (gd or gdj) else CHAIN_TOL
    for b, br in enumerate(ora.br):
        assert norm_rel(ctx.get_params(b), O.param_vec(br.weights, br.biases)) < ptol, b
        assert norm_rel(ctx.get_precisions(b), O.precision_vec(br)) < ptol, b
    assert norm_rel(net.residual(), ora.residual) < ptol
    assert abs(s["output_bias"] - ora.ob_bias) <= CHAIN_TOL * max(1.0, abs(ora.ob_bias))
    assert rel(s["error_precision"], ora.g_eprec) < CHAIN_TOL
    assert rel(s["output_reg_sum"], ora.g_reg) < CHAIN_TOL
    net.close()
    ctx.close()


def test_model_file_roundtrip(tmp_path):
    """models/<ix>.bin after burn-in + training_stats (net.rs:338-342, 565-569,
    train_stats.rs:83-87); the file parses as bincode Net<B> and loads back."""
    from bann import BannContext, MCMCConfig, Net
    ctx, branches, X, y = build("ridge_ard", seed=5)
    net = Net(ctx, seed=7)
    net.train(y, MCMCConfig(hmc_integration_length=5, chain_length=3), outdir=str(tmp_path))
    files = sorted(os.listdir(tmp_path / "models"))
    assert files == ["2.bin", "3.bin"], files   # burn_in = chain_length - 1 (mcmc_cfg.rs:152-156)
    f = NO.read_net_file(str(tmp_path / "models" / "3.bin"))
    s = net.summary()
    mse, lpd = net.records()
    assert f["num_branches"] == 3 and len(f["branch_cfgs"]) == 3
    assert f["hyperparams"]["output"] == {"shape": pytest.approx(0.001), "scale": pytest.approx(1000.0)}
    for b, cfg in enumerate(f["branch_cfgs"]):
        w = [np.asarray(v) for v in cfg["params"]["weights"]]
        bb = [np.asarray(v) for v in cfg["params"]["biases"]]
        assert np.array_equal(np.concatenate(w + bb).astype(np.float32), ctx.get_params(b))
        prec = cfg["precisions"]
        flat = np.concatenate([np.asarray(v) for v in prec["weight_precisions"]] +
                              [np.asarray(v) for v in prec["bias_precisions"]] + [np.asarray(prec["error_precision"])])
        assert np.array_equal(flat.astype(np.float32), ctx.get_precisions(b))
        assert cfg["num_params"] == ctx.num_params(b) and cfg["activation_function"] == 0
        assert cfg["layer_widths"] == cfg["params"]["layer_widths"] == list(branches[b].layer_widths)
        assert cfg["params"]["output_weight_summary_stats"]["num_params"] == 4 + 4 + 3
    ts = f["training_stats"]
    assert (ts["num_samples"], ts["num_accepted"], ts["num_early_rejected"]) == (
        s["num_samples"], s["num_accepted"], s["num_early_rejected"])
    assert np.array_equal(np.float32(ts["mse_train"]), mse) and np.array_equal(np.float32(ts["lpd"]), lpd)
    assert ts["mse_test"] is None
    gp = f["global_params"]
    assert gp["error_precision"] == pytest.approx(s["error_precision"], rel=1e-7)
    assert gp["output_weight_summary_stats"]["num_params"] == 11
    js = json.load(open(tmp_path / "training_stats"))
    assert js["num_samples"] == s["num_samples"] and len(js["lpd"]) == 4
    # load into a fresh context with the same branch shapes
    ctx2, _, _, _ = build("ridge_ard", seed=9)
    net2 = Net(ctx2)
    net2.load(str(tmp_path / "models" / "3.bin"))
    for b in range(3):
        assert np.array_equal(ctx2.get_params(b), ctx.get_params(b))
        assert np.array_equal(ctx2.get_precisions(b), ctx.get_precisions(b))
    s2 = net2.summary()
    for k in ("num_samples", "num_accepted", "num_records", "output_bias", "error_precision", "output_reg_sum"):
        assert s2[k] == s[k], k
    # a model whose shapes differ is refused
    ctx3, _, _, _ = build("ridge_ard", seed=9, ms=(40, 64, 31))
    net3 = Net(ctx3)
    from bann import BannError
    with pytest.raises(BannError):
        net3.load(str(tmp_path / "models" / "3.bin"))
    for o in (net, net2, net3, ctx, ctx2, ctx3):
        o.close()


def test_std_scaled_refused_for_ard():
    """StdScaled returns empty step sizes for the ARD priors (ridge_ard.rs:56-68,
    lasso_ard.rs:62-74) -- the reference's hmc_step would index-panic: the driver refuses
    the configuration before the first sweep."""
    from bann import BannError, MCMCConfig, Net
    ctx, branches, X, y = build("ridge_ard")
    net = Net(ctx, seed=3)
    with pytest.raises(BannError, match="ARD"):
        net.train(y, MCMCConfig(hmc_integration_length=5, chain_length=1, hmc_step_size_mode="std_scaled"))
    net.close()
    ctx.close()


def test_std_normal_cannot_train():
    """Net::train panics for StdNormalBranch (net.rs:167 -> std_normal_branch.rs:129);
    the driver refuses it at creation."""
    from bann import BannError, Net
    ctx, _, _, _ = build("std_normal")
    with pytest.raises(BannError):
        Net(ctx)
    ctx.close()


def test_training_reduces_mse():
    """built-in host RNG; the Izmailov sizes ignore the likelihood curvature
    (ridge_ard.rs:70-117), so at n = 3000 the step factor is lowered, as the
    reference's --hmc-step-size-factor (cli.rs:99-100) is used for."""
    from bann import MCMCConfig, Net
    ctx, _, _, y = build("ridge_ard", seed=21, n=3000)
    net = Net(ctx, seed=1)
    net.train(y, MCMCConfig(hmc_integration_length=20, chain_length=12, hmc_step_size_factor=0.1))
    mse, lpd = net.records()
    s = net.summary()
    assert s["num_samples"] == 36 and s["num_accepted"] > 0, s
    assert mse[-1] < mse[0], mse
    assert np.all(np.isfinite(lpd))
    net.close()
    ctx.close()


def test_trace_trajectories_and_test_mse(tmp_path):
    """f2: MCMCCfg::trace writes the BranchCfgs as one serde-JSON line after init
    and after every sweep (net.rs:241-244, 350-353); MCMCCfg::trajectories one
    Trajectory JSON per HMC step (trajectory.rs:3-11, branch_sampler.rs:1253-1289);
    a test set gives record_perf's mse_test (net.rs:597-610) in training_stats
    and in the model file."""
    from bann import BannContext, MCMCConfig, Net
    ctx, branches, X, y = build("ridge_ard", seed=5)
    rng = np.random.default_rng(77)
    ms = (40, 64, 30)
    gt = O.synthetic_genotypes(rng, 300, sum(ms))
    tctx = BannContext(0)
    tctx.upload_genotypes(gt)
    off = 0
    for m, br in zip(ms, branches):
        tctx.add_branch(np.arange(off, off + m, dtype=np.int32), br.layer_widths, "tanh", "ridge_ard")
        off += m
    tctx.finalize()
    y_test = rng.normal(size=300).astype(np.float32)
    net = Net(ctx, seed=3)
    net.set_test_data(tctx, y_test)
    L, chain = 4, 3
    net.train(y, MCMCConfig(hmc_integration_length=L, chain_length=chain, trace=True, trajectories=True),
              outdir=str(tmp_path))
    lines = open(tmp_path / "trace").read().splitlines()
    assert len(lines) == chain + 1
    last = json.loads(lines[-1])
    assert len(last) == 3 and last[0]["activation_function"] == "Tanh"
    for b, cfg in enumerate(last):
        w = [np.asarray(v, np.float32) for v in cfg["params"]["weights"]]
        bb = [np.asarray(v, np.float32) for v in cfg["params"]["biases"]]
        assert np.array_equal(np.concatenate(w + bb), ctx.get_params(b))
        assert cfg["num_params"] == ctx.num_params(b) and cfg["layer_widths"] == list(branches[b].layer_widths)
    trajs = [json.loads(t) for t in open(tmp_path / "traj").read().splitlines()]
    assert len(trajs) == chain * 3
    for t in trajs:
        k = len(t["params"])
        assert 1 <= k <= L and len(t["ldg"]) == k and len(t["hamiltonian"]) == k + 1
        assert t["precisions"] == [] and t["num_ldg"] == []
    mt = net.records_test()
    mse, _ = net.records()
    assert mt.size == mse.size == chain + 1
    mu, sd = tctx.genotype_stats()
    off, f = 0, np.zeros(300)
    for b, m in enumerate(ms):
        s = np.arange(off, off + m)
        off += m
        bw, bb = O.load_param_vec(ctx.get_params(b).astype(np.float64), m, branches[b].layer_widths)
        br = branches[b].copy()
        br.weights, br.biases = bw, bb
        f += O.predict(br, x_std(gt[s], mu[s], sd[s]))
    f += net.summary()["output_bias"]
    assert rel(float(mt[-1]), float(np.mean((y_test - f) ** 2))) < 1e-4
    js = json.load(open(tmp_path / "training_stats"))
    assert np.allclose(js["mse_test"], mt, rtol=1e-6)
    fm = NO.read_net_file(str(tmp_path / "models" / f"{chain}.bin"))
    assert np.array_equal(np.float32(fm["training_stats"]["mse_test"]), mt)
    for o in (net, ctx, tctx):
        o.close()


def test_joint_training_writes_joint_trajectories(tmp_path):
    """MCMCCfg::joint_hmc with MCMCCfg::trajectories: every hmc_step_joint writes
    the joint Trajectory line (branch_sampler.rs:1126-1135, early rejections
    included): per step the parameters, the precisions and the joint ldg
    [params | precisions], the joint -H trace; the chain itself stays the
    oracle's (recording does not change the launches' results)."""
    from bann import MCMCConfig, Net
    ctx, branches, X, y = build("ridge_ard")
    hp = O.Hyper()
    net = Net(ctx, (hp.dense, hp.summary, hp.output))
    d_dev, d_ora = NO.Draws(11), NO.Draws(11)
    net.set_rng(d_dev.uniform, d_dev.normal, d_dev.gamma)
    L, chain = 6, 2
    net.train(y, MCMCConfig(hmc_integration_length=L, chain_length=chain, hmc_step_size_factor=0.5, joint_hmc=True,
                            trajectories=True), outdir=str(tmp_path))
    trajs = [json.loads(t) for t in open(tmp_path / "traj").read().splitlines()]
    assert len(trajs) == chain * 3
    for t in trajs:
        k = len(t["params"])
        assert 1 <= k <= L and len(t["precisions"]) == k and len(t["ldg"]) == k and len(t["hamiltonian"]) == k + 1
        P = len(t["params"][0])
        Q = len(t["precisions"][0])
        assert P in [ctx.num_params(b) for b in range(3)] and Q > 0 and len(t["ldg"][0]) == P + Q
    ora = NO.NetOracle(branches, X, hp)
    ora.train(y.astype(np.float64), d_ora, chain, L, factor=0.5, joint_hmc=True)
    s = net.summary()
    assert (s["num_samples"], s["num_accepted"], s["num_early_rejected"]) == (ora.ns, ora.nacc, ora.nearly)
    for b, br in enumerate(ora.br):
        assert norm_rel(ctx.get_params(b), O.param_vec(br.weights, br.biases)) < CHAIN_TOL, b
    net.close()
    ctx.close()


def test_trajectory_recording_matches_oracle_hmc():
    """bann_set_trajectory_recording: the recorded parameters, gradients and -H of
    an injected-draw trajectory are the oracle's (params after each position
    step, ldg at them, the -H trace)."""
    from bann import BannContext
    ctx, branches, X, y = build("lasso_ard", seed=8)
    br = branches[0]
    ctx.set_target(0, y)
    L = 5
    ew, eb = O.izmailov_step_sizes(br, 0.5, L)
    eps = O.param_vec(ew, eb).astype(np.float32)
    p0 = np.random.default_rng(1).normal(size=br.num_params).astype(np.float32)
    ctx.set_trajectory_recording(True)
    res = ctx.hmc_step([0], L, 10.0, eps=eps, momentum=p0, u=[0.5])
    tr = ctx.get_trajectory(0)
    assert tr["params"].shape == (L, br.num_params) and tr["hamiltonian"].size == L + 1
    assert np.array_equal(tr["hamiltonian"], res["trace"][0])
    ob = br.copy()
    pw, pb = O.load_param_vec(p0.astype(np.float64), br.num_markers, br.layer_widths)
    ew2, eb2 = O.load_param_vec(eps.astype(np.float64), br.num_markers, br.layer_widths)
    th = O.param_vec(ob.weights, ob.biases)
    gw, gb, _ = O.log_density_gradient(ob, X[0], y.astype(np.float64))
    p = O.param_vec(pw, pb)
    e = O.param_vec(ew2, eb2)
    g = O.param_vec(gw, gb)
    for k in range(L):   # the oracle leapfrog, recording like branch_sampler.rs:1239-1262
        p = p + 0.5 * e * g
        th = th + e * p
        ob.weights, ob.biases = O.load_param_vec(th, br.num_markers, br.layer_widths)
        gw, gb, _ = O.log_density_gradient(ob, X[0], y.astype(np.float64))
        g = O.param_vec(gw, gb)
        p = p + 0.5 * e * g
        assert norm_rel(tr["params"][k], th) < 1e-5, k
        assert norm_rel(tr["ldg"][k], g) < 1e-5, k
    ctx.close()


def test_perturb_predict_and_test_data_checks():
    """Net::perturb (net.rs:187-199: + by to every param / precision), Net::predict
    (net.rs:545-559: bias + sum_b f_b, on the training cohort and on another
    cohort with the same branches), and bann_net_set_test_data refusing a
    y_test whose length is not the test cohort's."""
    from bann import BannContext, BannError, MCMCConfig, Net
    ctx, branches, X, y = build("ridge_ard", seed=13)
    net = Net(ctx, seed=2)
    net.train(y, MCMCConfig(hmc_integration_length=5, chain_length=2, hmc_step_size_factor=0.3))
    p0 = [ctx.get_params(b) for b in range(3)]
    q0 = [ctx.get_precisions(b) for b in range(3)]
    net.perturb(params_by=0.01)
    for b in range(3):
        assert np.array_equal(ctx.get_params(b), p0[b] + np.float32(0.01))
        assert np.array_equal(ctx.get_precisions(b), q0[b])
    net.perturb(precisions_by=0.5)
    for b in range(3):
        assert np.array_equal(ctx.get_precisions(b), q0[b] + np.float32(0.5))
    bias = net.summary()["output_bias"]
    f = np.zeros(y.size)
    for b in range(3):
        bw, bb = O.load_param_vec(ctx.get_params(b).astype(np.float64), branches[b].num_markers,
                                  branches[b].layer_widths)
        br = branches[b].copy()
        br.weights, br.biases = bw, bb
        f += O.predict(br, X[b])
    yh = net.predict()
    assert norm_rel(yh, f + bias) < 1e-5
    # another cohort with the same branches
    rng = np.random.default_rng(5)
    ms = (40, 64, 30)
    gt = O.synthetic_genotypes(rng, 250, sum(ms))
    tctx = BannContext(0)
    tctx.upload_genotypes(gt)
    off = 0
    for m, br in zip(ms, branches):
        tctx.add_branch(np.arange(off, off + m, dtype=np.int32), br.layer_widths, "tanh", "ridge_ard")
        off += m
    tctx.finalize()
    mu, sd = tctx.genotype_stats()
    ft, off = np.zeros(250), 0
    for b, m in enumerate(ms):
        s_ = np.arange(off, off + m)
        off += m
        bw, bb = O.load_param_vec(ctx.get_params(b).astype(np.float64), m, branches[b].layer_widths)
        br = branches[b].copy()
        br.weights, br.biases = bw, bb
        ft += O.predict(br, x_std(gt[s_], mu[s_], sd[s_]))
    assert norm_rel(net.predict(tctx), ft + bias) < 1e-5
    with pytest.raises(BannError):   # n_test must be the test cohort's size (it sizes the prediction buffer)
        net.set_test_data(tctx, np.zeros(100, np.float32))
    net.set_test_data(tctx, np.zeros(250, np.float32))
    for o in (net, ctx, tctx):
        o.close()


def test_net_gradient_r2s_rss_activations():
    """the other callers of the boundary: Net::gradient
    (net.rs:520-527: every branch's log_density_gradient against the phenotype,
    one packed launch), Net::branch_r2s (648-656, r2 = 1 - rss / sum y^2,
    branch_sampler.rs:911-913), Net::rss / mse (637-646) and Net::activations
    (509-518: forward_feed's activations of every layer) -- on the training
    context and on another cohort -- against the oracle."""
    from bann import BannContext, MCMCConfig, Net
    ctx, branches, X, y = build("ridge_ard", seed=12)
    net = Net(ctx, seed=4)
    net.train(y, MCMCConfig(hmc_integration_length=5, chain_length=2, hmc_step_size_factor=0.5))
    ms = (40, 64, 30)
    rng = np.random.default_rng(5)
    gt = O.synthetic_genotypes(rng, 500, sum(ms))
    tctx = BannContext(0)
    tctx.upload_genotypes(gt)
    off = 0
    for m, br in zip(ms, branches):
        tctx.add_branch(np.arange(off, off + m, dtype=np.int32), br.layer_widths, "tanh", "ridge_ard")
        off += m
    tctx.finalize()
    y_t = rng.normal(size=500).astype(np.float32)
    mu, sd = tctx.genotype_stats()
    Xt, off = [], 0
    for m in ms:
        s = np.arange(off, off + m)
        off += m
        Xt.append(x_std(gt[s], mu[s], sd[s]))
    oracle_brs = []
    for b, br in enumerate(branches):   # the net's current cfgs
        ob = br.copy()
        ob.weights, ob.biases = O.load_param_vec(ctx.get_params(b).astype(np.float64), br.num_markers, br.layer_widths)
        O.load_precision_vec(ob, ctx.get_precisions(b).astype(np.float64))
        oracle_brs.append(ob)
    for c, XX, yy in ((None, X, y), (tctx, Xt, y_t)):
        grads = net.gradient(yy, c)
        r2 = net.branch_r2s(yy, c)
        yd = yy.astype(np.float64)
        for b, ob in enumerate(oracle_brs):
            gw, gb, orss = O.log_density_gradient(ob, XX[b], yd)
            assert norm_rel(grads[b], O.param_vec(gw, gb)) < 1e-5, b
            assert abs(r2[b] - (1.0 - orss / float(yd @ yd))) <= 1e-5 * max(1.0, abs(r2[b])), b
            acts = net.activations(b, c)
            _, oacts = O.forward_feed(ob, XX[b])
            assert len(acts) == len(oacts)
            for a, oa in zip(acts, oacts):
                assert a.shape == oa.shape and norm_rel(a, oa) < 1e-5, b
        f = sum(O.predict(ob, xx) for ob, xx in zip(oracle_brs, XX)) + net.summary()["output_bias"]
        orss = float(np.sum((yd - f) ** 2))
        assert rel(net.rss(yy, c), orss) < 1e-5 and rel(net.mse(yy, c), orss / yy.size) < 1e-5
    for o in (net, ctx, tctx):
        o.close()
