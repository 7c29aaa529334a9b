"""GPU parity of the effect sizes (BranchSampler::effect_sizes,
branch_sampler.rs:784-811; Net::population_effect_sizes, net.rs:529-543; the
mcmc_cfg.effect_sizes CSV dump of Net::train, net.rs:307-315, 571-587) against
the float64 oracle (oracle/bann_oracle.py effect_sizes / population_effect_sizes).

Tolerance: norm-relative 1e-5 per matrix / vector (north_star).  The reference
seeds the chain with the branch output times W_out^T and takes no absolute
value; the oracle restates exactly that and is itself checked against a finite
difference of the prediction in tests/test_oracle_kats.py.
"""
import csv
import os

import numpy as np
import pytest

import bann_oracle as O
from helpers import build_context, f32_branch, norm_rel, x_std

pytestmark = pytest.mark.gpu
TOL = 1e-5

SHAPES = [("fx", 60, [4, 4, 1]), ("fxl", 700, [4, 3, 1]), ("wide", 40, [8, 8, 1]),
          ("layered", 30, [6, 5, 3, 1]), ("layered", 90, [45, 45, 1]), ("two-layer", 20, [3, 1])]


@pytest.fixture(scope="module")
def Ctx():
    from bann import BannContext
    return BannContext


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("act", ["tanh", "relu", "leaky_relu", "silu", "identity"])
def test_effect_sizes_match_oracle(Ctx, shape, act):
    """bann_effect_sizes: the n x m matrix of every kernel path's branch shapes."""
    _, m, widths = shape
    rng = np.random.default_rng(11)
    n = 333
    g = O.synthetic_genotypes(rng, n, m)
    br = f32_branch(O.random_branch(rng, m, widths, act=act))
    ctx = build_context(Ctx, g, [dict(snps=np.arange(m, dtype=np.int32), branch=br, y=np.zeros(n))])
    mu, sd = ctx.genotype_stats()
    X = x_std(g, mu, sd)
    e = ctx.effect_sizes(0)
    oe = O.effect_sizes(br, X)
    assert e.shape == oe.shape == (n, m)
    assert norm_rel(e, oe) < TOL
    ctx.close()


def test_population_effect_sizes(Ctx):
    """bann_population_effect_sizes: column means of each listed branch, in list
    order; equal (1e-5) to the oracle and to the column means of the full matrix."""
    rng = np.random.default_rng(5)
    n = 1000
    shapes = [(60, [4, 4, 1], "tanh"), (700, [4, 3, 1], "relu"), (40, [8, 8, 1], "silu"), (90, [45, 45, 1], "tanh")]
    g = O.synthetic_genotypes(rng, n, sum(m for m, _, _ in shapes))
    specs, off = [], 0
    for m, w, act in shapes:
        specs.append(dict(snps=np.arange(off, off + m, dtype=np.int32),
                          branch=f32_branch(O.random_branch(rng, m, w, act=act)), y=np.zeros(n)))
        off += m
    ctx = build_context(Ctx, g, specs)
    mu, sd = ctx.genotype_stats()
    Xs = [x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]]) for s in specs]
    order = [2, 0, 3, 1]
    pop = ctx.population_effect_sizes(order)
    opop = O.population_effect_sizes([specs[b]["branch"] for b in order], [Xs[b] for b in order])
    assert pop.shape == opop.shape
    at = 0
    for b in order:
        m = shapes[b][0]
        assert norm_rel(pop[at:at + m], opop[at:at + m]) < TOL, b
        assert norm_rel(pop[at:at + m], ctx.effect_sizes(b).astype(np.float64).mean(axis=0)) < TOL, b
        at += m
    ctx.close()


def rust_display(v: np.float32) -> str:
    """Rust's f32 Display: shortest round-trip digits, positional (numpy's Dragon4)."""
    return np.format_float_positional(np.float32(v), unique=True, trim="-")


def test_train_effect_size_csv_and_net_population(Ctx, tmp_path):
    """bann_net_train with effect_sizes: outdir/effect_sizes/<chain_ix>_<branch_ix>
    after burn-in (net.rs:307-315), one CSV row per individual (net.rs:571-587), the
    numbers as Rust prints an f32; the last sweep's files are effect_sizes at the final
    parameters.  bann_net_population_effect_sizes over the net's branches."""
    from bann.net import MCMCConfig, Net
    rng = np.random.default_rng(9)
    n = 300
    shapes = [(40, [4, 4, 1]), (30, [6, 3, 1])]
    g = O.synthetic_genotypes(rng, n, sum(m for m, _ in shapes))
    specs, off = [], 0
    for m, w in shapes:
        specs.append(dict(snps=np.arange(off, off + m, dtype=np.int32),
                          branch=f32_branch(O.random_branch(rng, m, w)), y=np.zeros(n)))
        off += m
    ctx = build_context(Ctx, g, specs)
    mu, sd = ctx.genotype_stats()
    Xs = [x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]]) for s in specs]
    y = rng.normal(size=n).astype(np.float32)
    net = Net(ctx, seed=3)
    cfg = MCMCConfig(hmc_step_size_factor=0.3, hmc_integration_length=5, chain_length=3, burn_in=2,
                     effect_sizes=True)
    net.train(y, cfg, outdir=str(tmp_path))
    files = sorted(os.listdir(tmp_path / "effect_sizes"))
    assert files == ["2_0", "2_1", "3_0", "3_1"], files
    finals = []
    for b, (m, w) in enumerate(shapes):
        br = O.Branch(m, list(w), prior=specs[b]["branch"].prior, act=specs[b]["branch"].act)
        br.weights, br.biases = O.load_param_vec(ctx.get_params(b).astype(np.float64), m, list(w))
        finals.append(br)
        with open(tmp_path / "effect_sizes" / f"3_{b}", newline="") as f:
            rows = list(csv.reader(f))
        assert len(rows) == n and all(len(r) == m for r in rows)
        vals = np.array([[np.float32(x) for x in r] for r in rows], np.float32)
        assert all(x == rust_display(v) for r, vr in zip(rows[:50], vals[:50]) for x, v in zip(r, vr))
        assert np.array_equal(vals, ctx.effect_sizes(b))
        assert norm_rel(vals, O.effect_sizes(br, Xs[b])) < TOL
    pop = net.population_effect_sizes()
    assert norm_rel(pop, O.population_effect_sizes(finals, Xs)) < TOL
    net.close()
    ctx.close()
