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


@pytest.mark.parametrize("prior,sampled_bias", [("ridge_ard", False), ("ridge_ard", True), ("lasso_base", False),
                                                ("lasso_ard", True)])
def test_train_matches_oracle(prior, sampled_bias):
    from bann import MCMCConfig, Net
    ctx, branches, X, y = build(prior)
    hp = O.Hyper()
    net = Net(ctx, (hp.dense, hp.summary, hp.output))
    d_dev, d_ora = NO.Draws(11), NO.Draws(11)
    net.set_rng(d_dev.uniform, d_dev.normal, d_dev.gamma)
    cfg = MCMCConfig(hmc_integration_length=10, chain_length=3, sampled_output_bias=sampled_bias)
    net.train(y, cfg)
    ora = NO.NetOracle(branches, X, hp)
    ora.train(y.astype(np.float64), d_ora, 3, 10, sampled_output_bias=sampled_bias)
    assert d_dev.uniform() == d_ora.uniform(), "draw streams diverged (different number of draws)"
    s = net.summary()
    assert (s["num_samples"], s["num_accepted"], s["num_early_rejected"]) == (ora.ns, ora.nacc, ora.nearly)
    mse, lpd = net.records()
    assert len(mse) == len(ora.mse) == 4
    for a, b in zip(mse, ora.mse):
        assert rel(a, b) < CHAIN_TOL, (mse, ora.mse)
    for a, b in zip(lpd, ora.lpd):
        assert rel(a, b) < CHAIN_TOL, (lpd, ora.lpd)
    for b, br in enumerate(ora.br):
        assert norm_rel(ctx.get_params(b), O.param_vec(br.weights, br.biases)) < CHAIN_TOL, b
        assert norm_rel(ctx.get_precisions(b), O.precision_vec(br)) < CHAIN_TOL, b
    assert norm_rel(net.residual(), ora.residual) < CHAIN_TOL
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
