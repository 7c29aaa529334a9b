"""Shared test utilities: build a device context and the matching oracle branch
on the SAME genotypes, standardization constants and parameters."""
from __future__ import annotations

import numpy as np

import bann_oracle as O


def norm_rel(a, b):
    a = np.asarray(a, dtype=np.float64).ravel()
    b = np.asarray(b, dtype=np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def x_std(g_block: np.ndarray, mu, sd) -> np.ndarray:
    """(n x m) standardized matrix from int8 [m][n] genotypes (bed.rs:325-355),
    float64; zero-variance markers -> 0 (documented deviation)."""
    g = g_block.astype(np.float64).T
    mu = np.asarray(mu, dtype=np.float64)
    sd = np.asarray(sd, dtype=np.float64)
    safe = np.where(sd > 0, sd, 1.0)
    x = (g - mu[None, :]) / safe[None, :]
    x[:, sd <= 0] = 0.0
    return x


def layer_views(br: O.Branch, vec: np.ndarray):
    """split a param_vec-ordered vector into per-layer weight and bias pieces."""
    return O.load_param_vec(np.asarray(vec, dtype=np.float64), br.num_markers, br.layer_widths)


def build_context(BannContext, g: np.ndarray, specs, fused=True, stats=None, free_raw=False):
    """specs: list of dicts {snps, branch (oracle Branch), y}.  Returns ctx."""
    ctx = BannContext(0)
    ctx.upload_genotypes(g)
    if stats is not None:
        ctx.set_genotype_stats(*stats)
    for s in specs:
        br = s["branch"]
        ctx.add_branch(s["snps"], br.layer_widths, br.act, br.prior)
    if not fused:
        ctx.set_fused_enabled(False)
    ctx.finalize(free_raw=free_raw)
    for b, s in enumerate(specs):
        br = s["branch"]
        ctx.set_params(b, O.param_vec(br.weights, br.biases))
        ctx.set_precisions(b, O.precision_vec(br))
        ctx.set_target(b, s["y"])
    return ctx


def f32_branch(br: O.Branch) -> O.Branch:
    """the branch with its parameters rounded to f32 (what the device holds),
    kept in float64 for the oracle."""
    b = br.copy()
    b.weights = [w.astype(np.float32).astype(np.float64) for w in b.weights]
    b.biases = [x.astype(np.float32).astype(np.float64) for x in b.biases]
    b.weight_precisions = [p.astype(np.float32).astype(np.float64) for p in b.weight_precisions]
    b.bias_precisions = [float(np.float32(x)) for x in b.bias_precisions]
    b.error_precision = float(np.float32(b.error_precision))
    return b
