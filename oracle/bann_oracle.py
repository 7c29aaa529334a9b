"""CPU oracle for the rs-bann branch HMC hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (the HIP library under
``rs-bann_amd/``) may import or call this module; only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it, and
only as the checker.

This is a numpy restatement of the reference's (medical-genomics-group/rs-bann,
Rust + ArrayFire 3.8) per-branch math.  Every function cites the reference
file:line it follows (paths relative to the reference repo root).

Parity pinning: the restatement is checked against the reference's own
known-answer tests (``tests/golden/reference_kats.json``, transcribed from
``src/net/branch/{ridge_ard,ridge_base,lasso_ard,lasso_base}.rs`` tests and
``src/io/bed.rs`` tests) and against ``py-vis/sim.py`` generated vectors
(``tests/golden/sim_py_vectors.json``).  See ``tests/test_oracle_kats.py``.

Layout conventions (reference, ArrayFire column-major):
  * weights[l] is an (in_l x out_l) matrix; the flat/param-vector order is
    column-major: element (j, k) at k * in_l + j.
  * biases[l] is a length out_l row vector, for l in 0..num_layers-2 (the
    output neuron has no bias).
  * X is (n x m) individuals x markers, standardized.

``dtype`` selects the arithmetic type: float64 is the "truth" used by the
parity tests; float32 mimics the reference's single precision arithmetic.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

# Activation codes follow the enum order of src/net/activation_functions.rs:6-12
ACTIVATIONS = {"tanh": 0, "relu": 1, "leaky_relu": 2, "silu": 3, "identity": 4}
# Prior codes (one per BranchSampler impl, src/net/branch/*.rs)
PRIORS = {"ridge_ard": 0, "ridge_base": 1, "lasso_ard": 2, "lasso_base": 3, "std_normal": 4}
ARD_PRIORS = ("ridge_ard", "lasso_ard")


# --------------------------------------------------------------------------
# activations: src/net/activation_functions.rs:22-45
# --------------------------------------------------------------------------
def _afsign(x):
    """ArrayFire ``sign``: 1 for negative values, 0 otherwise."""
    return (x < 0).astype(x.dtype)


def h(x: np.ndarray, act: str) -> np.ndarray:
    """activation_functions.rs:23-30"""
    if act == "tanh":
        return np.tanh(x)
    if act == "relu":
        return x * (x > 0).astype(x.dtype)
    if act == "leaky_relu":
        return x * (x > 0).astype(x.dtype) + x * _afsign(x) * x.dtype.type(0.01)
    if act == "silu":
        return x * (1.0 / (1.0 + np.exp(-x))).astype(x.dtype)
    if act == "identity":
        return x.copy()
    raise ValueError(act)


def dhdx(x: np.ndarray, act: str) -> np.ndarray:
    """activation_functions.rs:32-44"""
    if act == "tanh":
        t = np.tanh(x)
        return 1 - t * t
    if act == "relu":
        return (x > 0).astype(x.dtype)
    if act == "leaky_relu":
        return (x > 0).astype(x.dtype) + _afsign(x) * x.dtype.type(0.01)
    if act == "silu":
        s = (1.0 / (1.0 + np.exp(-x))).astype(x.dtype)
        fx = x * s
        return fx + s * (1 - fx)
    if act == "identity":
        return np.ones_like(x)
    raise ValueError(act)


def af_sign(x: np.ndarray) -> np.ndarray:
    """af_helpers.rs:53-58: 0 - afsign(x) + (x > 0)  ==  -1 / 0 / +1."""
    return np.sign(x)


# --------------------------------------------------------------------------
# branch state: src/net/params.rs:192-199 (precisions), 468-476 / 619-625 (params)
# --------------------------------------------------------------------------
@dataclass
class Branch:
    num_markers: int
    layer_widths: List[int]            # hidden..., summary, 1 (params.rs:470)
    prior: str = "ridge_ard"
    act: str = "tanh"
    weights: List[np.ndarray] = field(default_factory=list)   # (in, out)
    biases: List[np.ndarray] = field(default_factory=list)    # (out,)
    weight_precisions: List[np.ndarray] = field(default_factory=list)
    bias_precisions: List[float] = field(default_factory=list)
    error_precision: float = 1.0
    # OutputWeightSummaryStats (params.rs:404-465): reg sum of the OTHER branches'
    # output weights and the global output-weight count.
    out_reg_sum: float = 0.0
    out_num_params: Optional[float] = None

    @property
    def num_layers(self) -> int:
        return len(self.layer_widths)

    @property
    def output_layer_index(self) -> int:
        return self.num_layers - 1

    def in_width(self, l: int) -> int:
        return self.num_markers if l == 0 else self.layer_widths[l - 1]

    @property
    def num_params(self) -> int:
        """branch_cfg_builder.rs:123-128,285-297"""
        return sum(w.size for w in self.weights) + sum(b.size for b in self.biases)

    def copy(self) -> "Branch":
        return Branch(
            self.num_markers, list(self.layer_widths), self.prior, self.act,
            [w.copy() for w in self.weights], [b.copy() for b in self.biases],
            [p.copy() for p in self.weight_precisions], list(self.bias_precisions),
            self.error_precision, self.out_reg_sum, self.out_num_params)

    def astype(self, dtype) -> "Branch":
        b = self.copy()
        b.weights = [w.astype(dtype) for w in b.weights]
        b.biases = [x.astype(dtype) for x in b.biases]
        b.weight_precisions = [p.astype(dtype) for p in b.weight_precisions]
        return b


def param_vec(weights: Sequence[np.ndarray], biases: Sequence[np.ndarray]) -> np.ndarray:
    """params.rs:700-715: all weights (column-major, layer order), then all biases."""
    parts = [np.asarray(w).reshape(-1, order="F") for w in weights]
    parts += [np.asarray(b).reshape(-1) for b in biases]
    return np.concatenate(parts) if parts else np.zeros(0)


def load_param_vec(vec: np.ndarray, num_markers: int, layer_widths: Sequence[int]):
    """params.rs:673-698 (inverse of param_vec)."""
    weights, biases = [], []
    prev, ix = num_markers, 0
    for w in layer_widths:
        weights.append(np.asarray(vec[ix:ix + prev * w]).reshape((prev, w), order="F").copy())
        ix += prev * w
        prev = w
    for w in layer_widths[:-1]:
        biases.append(np.asarray(vec[ix:ix + w]).copy())
        ix += w
    return weights, biases


def precision_vec(br: Branch) -> np.ndarray:
    """params.rs:272-289: weight precisions (layer order), bias precisions, error precision."""
    parts = [np.asarray(p, dtype=np.float64).reshape(-1) for p in br.weight_precisions]
    parts.append(np.asarray(br.bias_precisions, dtype=np.float64))
    parts.append(np.asarray([br.error_precision], dtype=np.float64))
    return np.concatenate(parts)


# --------------------------------------------------------------------------
# forward / backward: src/net/branch/branch_sampler.rs:743-875
# --------------------------------------------------------------------------
def forward_feed(br: Branch, X: np.ndarray):
    """branch_sampler.rs:743-782. Returns (pre_activations, activations)."""
    L = br.num_layers
    pre = [X @ br.weights[0] + br.biases[0][None, :]]              # 760-773
    acts = [h(pre[-1], br.act)]
    for l in range(1, L - 1):                                        # 750-754
        pre.append(acts[-1] @ br.weights[l] + br.biases[l][None, :])
        acts.append(h(pre[-1], br.act))
    acts.append(acts[-1] @ br.weights[L - 1])                        # 775-782 (no bias)
    return pre, acts


def predict(br: Branch, X: np.ndarray) -> np.ndarray:
    """branch_sampler.rs:915-918"""
    return forward_feed(br, X)[1][-1][:, 0]


def rss(br: Branch, X: np.ndarray, y: np.ndarray) -> float:
    """branch_sampler.rs:905-909"""
    r = predict(br, X) - y
    return float(np.sum(r * r))


def backpropagate(br: Branch, X: np.ndarray, y: np.ndarray):
    """branch_sampler.rs:813-875 (half-rss gradient: error seeded with pred - y).

    Returns (rss, d_rss_wrt_weights, d_rss_wrt_biases).
    """
    L = br.num_layers
    pre, acts = forward_feed(br, X)
    err = acts[-1] - y.reshape(-1, 1)                                # 821
    rss_v = float(np.sum(err * err))                                  # 823-828
    dW = [None] * L
    db = [None] * (L - 1)
    dW[L - 1] = acts[L - 2].T @ err                                   # 830-835
    err = err @ br.weights[L - 1].T                                   # 837-842
    for l in range(L - 2, 0, -1):                                     # 844-859
        delta = dhdx(pre[l], br.act) * err
        db[l] = delta.sum(axis=0)
        dW[l] = acts[l - 1].T @ delta
        err = delta @ br.weights[l].T
    delta = dhdx(pre[0], br.act) * err                                # 861-866
    db[0] = delta.sum(axis=0)
    dW[0] = X.T @ delta
    return rss_v, dW, db


def effect_sizes(br: Branch, X: np.ndarray) -> np.ndarray:
    """branch_sampler.rs:784-811: out_i d out_i / d x_ij per individual and marker (n x m).

    As the reference computes it: the chain is seeded with the branch OUTPUT
    times W_out^T (792-797), not with the error, and no absolute value is taken
    (the doc comment says "absolute values"; the code does not)."""
    L = br.num_layers
    pre, acts = forward_feed(br, X)                                   # 789
    err = acts[-1] @ br.weights[L - 1].T                              # 792-797
    for l in range(L - 2, -1, -1):                                    # 799-808
        delta = dhdx(pre[l], br.act) * err
        err = delta @ br.weights[l].T
    return err


def population_effect_sizes(branches: Sequence[Branch], Xs: Sequence[np.ndarray]) -> np.ndarray:
    """net.rs:529-543: per branch the column sums of effect_sizes / n, concatenated."""
    return np.concatenate([effect_sizes(br, X).sum(axis=0) / X.shape[0] for br, X in zip(branches, Xs)])


# --------------------------------------------------------------------------
# priors: log density and gradient w.r.t. weights
# --------------------------------------------------------------------------
def _row_sumsq(w):
    return np.sum(w * w, axis=1)


def _row_l1(w):
    return np.sum(np.abs(w), axis=1)


def ldg_wrt_weights(br: Branch, dW) -> List[np.ndarray]:
    """Prior-specific gradient of the log density w.r.t. the weights.

    ridge_ard.rs:196-219, ridge_base.rs:175-184, lasso_ard.rs:196-218,
    lasso_base.rs:175-185, std_normal_branch.rs:160-169.
    """
    le = br.error_precision
    out = []
    L = br.num_layers
    for l in range(L):
        w = br.weights[l]
        lam = np.asarray(br.weight_precisions[l]) if br.weight_precisions else None
        if br.prior == "std_normal":
            reg = w
        elif br.prior in ARD_PRIORS and l < L - 1:
            lam_m = lam.reshape(-1, 1)                      # tile over columns
            reg = lam_m * (w if br.prior == "ridge_ard" else af_sign(w))
        else:
            lam_s = lam.reshape(-1)[0]
            reg = lam_s * (w if br.prior.startswith("ridge") else af_sign(w))
        out.append(-(le * dW[l] + reg))
    return out


def ldg_wrt_biases(br: Branch, db) -> List[np.ndarray]:
    """branch_sampler.rs:322-331 (unregularized biases)."""
    return [-br.error_precision * d for d in db]


def log_density_gradient(br: Branch, X, y):
    """branch_sampler.rs:380-391. Returns (grad_w, grad_b, rss)."""
    r, dW, db = backpropagate(br, X, y)
    return ldg_wrt_weights(br, dW), ldg_wrt_biases(br, db), r


def log_density_wrt_weights(br: Branch) -> float:
    """ridge_ard.rs:171-194, ridge_base.rs:154-166, lasso_ard.rs:171-194,
    lasso_base.rs:160-172, std_normal_branch.rs:138-147."""
    L = br.num_layers
    ld = 0.0
    for l in range(L):
        w = br.weights[l]
        if br.prior == "std_normal":
            ld -= float(np.sum(w * w)) / 2.0
            continue
        lam = np.asarray(br.weight_precisions[l]).reshape(-1)
        ridge = br.prior.startswith("ridge")
        if br.prior in ARD_PRIORS and l < L - 1:
            stat = _row_sumsq(w) * 0.5 if ridge else _row_l1(w)
            ld -= float(np.dot(stat, lam))
        else:
            stat = 0.5 * float(np.sum(w * w)) if ridge else float(np.sum(np.abs(w)))
            ld -= stat * float(lam[0])
    return ld


def log_density_wrt_rss(br: Branch, rss_v: float) -> float:
    """branch_sampler.rs:100-102"""
    return -br.error_precision * (rss_v / 2.0)


def log_density(br: Branch, rss_v: float) -> float:
    """branch_sampler.rs:72-78 (biases unregularized, 106-112); std_normal overrides
    (std_normal_branch.rs:149-158) with an L2 bias term."""
    if br.prior == "std_normal":
        ld = -0.5 * br.error_precision * rss_v
        for w in br.weights:
            ld -= 0.5 * float(np.sum(w * w))
        for b in br.biases:
            ld -= 0.5 * float(np.sum(b * b))
        return ld
    return log_density_wrt_weights(br) + log_density_wrt_rss(br, rss_v)


# --------------------------------------------------------------------------
# joint log density / gradient (precisions as parameters)
# --------------------------------------------------------------------------
@dataclass
class Hyper:
    """NetworkPrecisionHyperparameters (params.rs:134-188)."""
    dense: tuple = (0.001, 1000.0)
    summary: tuple = (0.001, 1000.0)
    output: tuple = (0.001, 1000.0)

    def layer(self, l: int, L: int):
        """params.rs:146-163"""
        if l == L - 1:
            return self.output
        if l == L - 2:
            return self.summary
        return self.dense


def ld_joint_wrt_rss(br: Branch, rss_v: float, hp: Hyper, n: int) -> float:
    """branch_sampler.rs:240-257"""
    k, s = hp.output
    le = br.error_precision
    return (k + (n - 2.0) / 2.0) * math.log(le) - le * (rss_v / 2.0 + 1.0 / s)


def ld_joint_wrt_biases(br: Branch, hp: Hyper) -> float:
    """branch_sampler.rs:260-279"""
    L = br.num_layers
    ld = 0.0
    for i in range(L - 1):
        shape, scale = hp.layer(i, L)
        lam = br.bias_precisions[i]
        b = br.biases[i]
        ld -= lam * (float(np.sum(b * b)) / 2.0 + 1.0 / scale)
        ld += (shape + (b.size - 2.0) / 2.0) * math.log(lam)
    return ld


def _out_num_params(br: Branch) -> float:
    if br.out_num_params is not None:
        return br.out_num_params
    return float(br.weights[-1].size)


def ld_joint_wrt_local_weights(br: Branch, hp: Hyper) -> float:
    """ridge_ard.rs:119-148, ridge_base.rs:119-137, lasso_ard.rs:119-149, lasso_base.rs:119-137"""
    L = br.num_layers
    ld = 0.0
    for i in range(L - 1):
        shape, scale = hp.layer(i, L)
        w = br.weights[i]
        lam = np.asarray(br.weight_precisions[i], dtype=np.float64).reshape(-1)
        nrows, ncols = w.shape
        if br.prior == "ridge_ard":
            ld -= float(np.dot(_row_sumsq(w) / 2.0 + 1.0 / scale, lam))
            ld += float(np.sum((shape + (ncols - 2.0) / 2.0) * np.log(lam)))
        elif br.prior == "lasso_ard":
            ld -= float(np.dot(_row_l1(w) + 1.0 / scale, lam))
            ld += float(np.sum((shape + ncols - 1.0) * np.log(lam)))
        elif br.prior == "ridge_base":
            ld -= (float(np.sum(w * w)) / 2.0 + 1.0 / scale) * lam[0]
            ld += (shape + (w.size - 2.0) / 2.0) * math.log(lam[0])
        elif br.prior == "lasso_base":
            ld -= (float(np.sum(np.abs(w))) + 1.0 / scale) * lam[0]
            ld += (shape + w.size - 1.0) * math.log(lam[0])
        else:
            raise NotImplementedError("std_normal has no joint density (std_normal_branch.rs:119-131)")
    return ld


def ld_joint_wrt_output_weights(br: Branch, hp: Hyper) -> float:
    """ridge_ard.rs:150-169 (ridge_base identical), lasso_ard.rs:151-169 (lasso_base identical)."""
    L = br.num_layers
    shape, scale = hp.layer(L - 1, L)
    w = br.weights[L - 1]
    lam = float(np.asarray(br.weight_precisions[L - 1]).reshape(-1)[0])
    npar = _out_num_params(br)
    if br.prior.startswith("ridge"):
        gss = float(np.sum(w * w)) + br.out_reg_sum
        return -((0.5 * gss) + 1.0 / scale) * lam + (shape + (npar - 2.0) / 2.0) * math.log(lam)
    if br.prior.startswith("lasso"):
        gsa = float(np.sum(np.abs(w))) + br.out_reg_sum
        return -(gsa + 1.0 / scale) * lam + (shape + npar - 1.0) * math.log(lam)
    raise NotImplementedError("std_normal")


def ld_joint_wrt_weights(br: Branch, hp: Hyper) -> float:
    """branch_sampler.rs:229-237"""
    return ld_joint_wrt_local_weights(br, hp) + ld_joint_wrt_output_weights(br, hp)


def log_density_joint(br: Branch, rss_v: float, hp: Hyper, n: int) -> float:
    """branch_sampler.rs:292-305"""
    return ld_joint_wrt_weights(br, hp) + ld_joint_wrt_biases(br, hp) + ld_joint_wrt_rss(br, rss_v, hp, n)


def ldg_joint(br: Branch, X, y, hp: Hyper):
    """branch_sampler.rs:406-422 with 333-378 and the prior-specific
    log_density_gradient_wrt_weight_precisions (ridge_ard.rs:221-250 etc.)."""
    r, dW, db = backpropagate(br, X, y)
    L = br.num_layers
    gw = ldg_wrt_weights(br, dW)
    gb = [-br.bias_precisions[i] * br.biases[i] - br.error_precision * db[i] for i in range(L - 1)]
    gwp = []
    for i in range(L - 1):
        shape, scale = hp.layer(i, L)
        w = br.weights[i]
        lam = np.asarray(br.weight_precisions[i], dtype=np.float64).reshape(-1)
        if br.prior == "ridge_ard":   # quirk: lam.size (rows), SURVEY App. B quirk 1
            gwp.append((2 * shape + lam.size - 2.0) / (2 * lam) - 1.0 / scale - _row_sumsq(w) / 2.0)
        elif br.prior == "lasso_ard":
            gwp.append((shape + lam.size - 1.0) / lam - 1.0 / scale - _row_l1(w))
        elif br.prior == "ridge_base":
            gwp.append(np.array([(2 * shape + w.size - 2.0) / (2 * lam[0]) - 1.0 / scale - np.sum(w * w) / 2.0]))
        elif br.prior == "lasso_base":
            gwp.append(np.array([(shape + w.size - 1.0) / lam[0] - 1.0 / scale - np.sum(np.abs(w))]))
        else:
            raise NotImplementedError
    shape, scale = hp.layer(L - 1, L)
    w = br.weights[L - 1]
    lam = float(np.asarray(br.weight_precisions[L - 1]).reshape(-1)[0])
    npar = _out_num_params(br)
    if br.prior.startswith("ridge"):
        gwp.append(np.array([(2 * shape + npar - 2.0) / (2 * lam) - 1.0 / scale
                             - (np.sum(w * w) + br.out_reg_sum) / 2.0]))
    else:
        gwp.append(np.array([(shape + npar - 1.0) / lam - 1.0 / scale - (np.sum(np.abs(w)) + br.out_reg_sum)]))
    gbp = []
    for i in range(L - 1):
        shape, scale = hp.layer(i, L)
        lam = br.bias_precisions[i]
        b = br.biases[i]
        gbp.append((2 * shape + (b.size - 2.0)) / (2 * lam) - 1.0 / scale - np.sum(b * b) / 2.0)
    k, s = hp.output
    n = y.size
    gep = (2 * k + n - 2.0) / (2 * br.error_precision) - 1.0 / s - r / 2.0
    return dict(wrt_weights=gw, wrt_biases=gb, wrt_weight_precisions=gwp,
                wrt_bias_precisions=gbp, wrt_error_precision=gep, rss=r)


# --------------------------------------------------------------------------
# step sizes: branch_sampler.rs:654-737, ridge_ard.rs:70-117 and siblings
# --------------------------------------------------------------------------
def izmailov_step_sizes(br: Branch, c: float, L_int: int):
    """Izmailov step sizes (default StepSizeMode, mcmc_cfg.rs:39).

    ridge_ard.rs:70-117, ridge_base.rs:83-114, lasso_ard.rs:77-117,
    lasso_base.rs:83-114, std_normal_branch.rs:83-114.
    Returns (eps_w, eps_b) as full-shape arrays.
    """
    L = br.num_layers
    eps_w, eps_b = [], []
    for l in range(L):
        w = br.weights[l]
        lam = np.asarray(br.weight_precisions[l], dtype=np.float64).reshape(-1)
        if br.prior == "std_normal":
            e = math.pi / (2 * math.sqrt(lam[0]) * L_int) * np.ones(w.shape)
        elif br.prior in ARD_PRIORS and l < L - 1:
            if br.prior == "ridge_ard":
                row = c * math.pi / (2 * np.sqrt(lam) * L_int)
            else:
                row = c * 1.0 / (4 * lam * L_int)
            e = np.tile(row.reshape(-1, 1), (1, w.shape[1]))
        else:
            if br.prior.startswith("ridge"):
                e = c * math.pi / (2 * math.sqrt(lam[0]) * L_int) * np.ones(w.shape)
            else:
                e = c / (4 * lam[0] * L_int) * np.ones(w.shape)
        eps_w.append(e)
    for l in range(L - 1):
        lamb = br.bias_precisions[l]
        cc = 1.0 if br.prior == "std_normal" else c
        eps_b.append(cc * math.pi / (2 * math.sqrt(lamb) * L_int) * np.ones(br.biases[l].shape))
    return eps_w, eps_b


def std_scaled_step_sizes(br: Branch, c: float):
    """StdScaled step sizes (StepSizeMode::StdScaled, dispatched at branch_sampler.rs:1213).

    ridge_base.rs:52-82, lasso_base.rs:53-82, std_normal_branch.rs:51-80, in f32 as the
    reference computes them: weights c * (1 / lambda_l).sqrt() (a host f32 scalar),
    biases c * (1 / sqrt(lambda_b)) (ArrayFire f32; lasso_base's 1 * c * (1 / sqrt) is the
    same value).  The ARD priors return EMPTY vectors (ridge_ard.rs:56-68,
    lasso_ard.rs:62-74), on which the reference's leapfrog index-panics: ValueError here.
    Returns (eps_w, eps_b) as full-shape float32 arrays."""
    if br.prior in ARD_PRIORS:
        raise ValueError("StdScaled step sizes are empty for the ARD priors (ridge_ard.rs:56-68)")
    f32 = np.float32
    cc = f32(c)
    eps_w = []
    for l in range(br.num_layers):
        lam = f32(np.asarray(br.weight_precisions[l], dtype=np.float32).reshape(-1)[0])
        e = f32(cc * np.sqrt(f32(f32(1.0) / lam), dtype=np.float32))
        eps_w.append(np.full(br.weights[l].shape, e, dtype=np.float32))
    eps_b = []
    for l in range(br.num_layers - 1):
        lamb = f32(np.asarray(br.bias_precisions[l], dtype=np.float32).reshape(-1)[0])
        e = f32(cc * f32(f32(1.0) / np.sqrt(lamb, dtype=np.float32)))
        eps_b.append(np.full(br.biases[l].shape, e, dtype=np.float32))
    return eps_w, eps_b


def uniform_step_sizes(br: Branch, c: float):
    """branch_sampler.rs:706-732"""
    return [c * np.ones(w.shape) for w in br.weights], [c * np.ones(b.shape) for b in br.biases]


def random_step_sizes(br: Branch, c: float, u_w, u_b):
    """branch_sampler.rs:654-681 with injected uniforms (ArrayFire randu is unseeded)."""
    f = br.num_params ** -0.25 * c
    return [f * np.asarray(u) for u in u_w], [f * np.asarray(u) for u in u_b]


# --------------------------------------------------------------------------
# momentum / leapfrog: momentum.rs:121-158, params.rs:728-738
# --------------------------------------------------------------------------
def kinetic(p_w, p_b) -> float:
    """momentum.rs:149-158: K(p) = p^T p / 2"""
    return 0.5 * (sum(float(np.sum(p * p)) for p in p_w) + sum(float(np.sum(p * p)) for p in p_b))


def neg_hamiltonian(br: Branch, p_w, p_b, X, y) -> float:
    """branch_sampler.rs:878-883"""
    return log_density(br, rss(br, X, y)) - kinetic(p_w, p_b)


def net_movement(br: Branch, init: Branch, p_w, p_b) -> float:
    """branch_sampler.rs:551-588: sum over layers of <theta - theta0, p>."""
    s = 0.0
    for l in range(br.num_layers):
        s += float(np.sum((br.weights[l] - init.weights[l]) * p_w[l]))
    for l in range(br.num_layers - 1):
        s += float(np.sum((br.biases[l] - init.biases[l]) * p_b[l]))
    return s


ACCEPTED, REJECTED, REJECTED_EARLY = 0, 1, 2


def hmc_step(br: Branch, X, y, eps_w, eps_b, p_w, p_b, L_int: int, max_dH: float, u: float):
    """branch_sampler.rs:1192-1299 + accept_or_reject_hmc_state 928-962.

    RNG draws are injected (momentum p, step sizes eps, acceptance uniform u),
    the parity protocol of SURVEY §0 caveat 3.  ``br`` is updated in place.
    Returns a dict with status, the H trace, the U-turn step and, if accepted,
    y_pred and log_density.
    """
    init = br.copy()
    p_w = [np.array(p, dtype=np.float64) for p in p_w]
    p_b = [np.array(p, dtype=np.float64) for p in p_b]
    H0 = neg_hamiltonian(br, p_w, p_b, X, y)                          # 1224
    gw, gb, _ = log_density_gradient(br, X, y)                         # 1232-1236
    trace = [H0]
    u_turn_step = -1
    for step in range(L_int):                                          # 1239
        for l in range(len(p_w)):                                      # half_step
            p_w[l] += 0.5 * eps_w[l] * gw[l]
        for l in range(len(p_b)):
            p_b[l] += eps_b[l] * 0.5 * gb[l]
        for l in range(len(p_w)):                                      # full_step
            br.weights[l] = br.weights[l] + eps_w[l] * p_w[l]
        for l in range(len(p_b)):
            br.biases[l] = br.biases[l] + eps_b[l] * p_b[l]
        gw, gb, _ = log_density_gradient(br, X, y)                     # 1243-1247
        for l in range(len(p_w)):                                      # 1249
            p_w[l] += 0.5 * eps_w[l] * gw[l]
        for l in range(len(p_b)):
            p_b[l] += eps_b[l] * 0.5 * gb[l]
        H = neg_hamiltonian(br, p_w, p_b, X, y)                         # 1253
        trace.append(H)
        if abs(H - H0) > max_dH:                                       # 1264-1279
            br.weights, br.biases = init.weights, init.biases
            return dict(status=REJECTED_EARLY, trace=trace, step=step, u_turn_step=u_turn_step)
        if u_turn_step < 0 and net_movement(br, init, p_w, p_b) < 0.0:  # 1281-1284
            u_turn_step = step
    y_pred = predict(br, X)                                            # 940-950
    r = y_pred - y
    ld = log_density(br, float(np.sum(r * r)))
    log_acc = (ld - kinetic(p_w, p_b)) - H0
    acc_p = 1.0 if log_acc >= 0 else math.exp(log_acc)
    if u < acc_p:
        return dict(status=ACCEPTED, trace=trace, y_pred=y_pred, log_density=ld,
                    u_turn_step=u_turn_step, p_w=p_w, p_b=p_b)
    br.weights, br.biases = init.weights, init.biases
    return dict(status=REJECTED, trace=trace, u_turn_step=u_turn_step, p_w=p_w, p_b=p_b)


# --------------------------------------------------------------------------
# joint HMC over parameters and precisions: branch_sampler.rs:1070-1178
# --------------------------------------------------------------------------
def load_precision_vec(br: Branch, vec) -> None:
    """inverse of precision_vec (params.rs:272-289), in place."""
    vec = np.asarray(vec, dtype=np.float64)
    ix, wp = 0, []
    for p in br.weight_precisions:
        shp = np.asarray(p).shape
        k = int(np.prod(shp)) if shp else 1
        wp.append(vec[ix:ix + k].reshape(shp).copy())
        ix += k
    nb = len(br.bias_precisions)
    br.weight_precisions = wp
    br.bias_precisions = [float(v) for v in vec[ix:ix + nb]]
    br.error_precision = float(vec[ix + nb])


def ldg_joint_vec(br: Branch, X, y, hp: Hyper):
    """log_density_gradient_joint (branch_sampler.rs:406-422) as one vector:
    [param_vec order | precision_vec order], and the rss."""
    g = ldg_joint(br, X, y, hp)
    gph = [np.asarray(x, dtype=np.float64).reshape(-1) for x in g["wrt_weight_precisions"]]
    gph += [np.asarray(g["wrt_bias_precisions"], dtype=np.float64).reshape(-1),
            np.asarray([g["wrt_error_precision"]], dtype=np.float64)]
    return np.concatenate([param_vec(g["wrt_weights"], g["wrt_biases"])] + gph), g["rss"]


def hmc_step_joint(br: Branch, X, y, hp: Hyper, eps, p, L_int: int, max_dH: float, u: float):
    """hmc_step_joint (branch_sampler.rs:1070-1178): leapfrog over the parameters
    AND the precisions (params.full_step + precisions.full_step, 1116-1117), -H
    from log_density_joint (886-901), early rejection on the joint -H, then
    accept_or_reject_hmc_state (928-962), whose final -H uses the NON-joint
    log_density -- a reference quirk reproduced here.  eps, p: concatenated
    [param_vec | precision_vec] step sizes and momenta (injected draws).
    ``br`` is updated in place (restored on rejection)."""
    n = y.size
    P = br.num_params
    init = br.copy()
    eps = np.asarray(eps, dtype=np.float64)
    p = np.array(p, dtype=np.float64)

    def state():
        return np.concatenate([param_vec(br.weights, br.biases), precision_vec(br)])

    def set_state(v):
        br.weights, br.biases = load_param_vec(v[:P], br.num_markers, br.layer_widths)
        load_precision_vec(br, v[P:])

    def neg_h():
        with np.errstate(all="ignore"):
            return log_density_joint(br, rss(br, X, y), hp, n) - 0.5 * float(p @ p)

    H0 = neg_h()
    g, _ = ldg_joint_vec(br, X, y, hp)
    trace = [H0]
    states, ldgs = [], []   # the joint Trajectory (1126-1135): state and ldg after every step
    for step in range(L_int):
        p += 0.5 * eps * g                                             # 1114
        set_state(state() + eps * p)                                   # 1115-1116
        with np.errstate(all="ignore"):
            g, _ = ldg_joint_vec(br, X, y, hp)                         # 1118
        p += 0.5 * eps * g                                             # 1119
        H = neg_h()                                                    # 1123-1124
        trace.append(H)
        states.append(state())
        ldgs.append(g.copy())
        if abs(H - H0) > max_dH:                                       # 1138-1158 (NaN never exceeds)
            br.weights, br.biases = init.weights, init.biases
            load_precision_vec(br, precision_vec(init))
            return dict(status=REJECTED_EARLY, trace=trace, step=step, states=states, ldgs=ldgs)
    r = predict(br, X) - y
    with np.errstate(all="ignore"):
        ld = log_density(br, float(np.sum(r * r)))                     # non-joint (943)
        log_acc = (ld - 0.5 * float(p @ p)) - H0
        acc_p = 1.0 if log_acc >= 0 else math.exp(log_acc)
    if u < acc_p:
        return dict(status=ACCEPTED, trace=trace, log_density=ld, p=p, states=states, ldgs=ldgs)
    br.weights, br.biases = init.weights, init.biases
    load_precision_vec(br, precision_vec(init))
    return dict(status=REJECTED, trace=trace, log_density=ld, p=p, states=states, ldgs=ldgs)


def gradient_descent(br: Branch, X, y, factor: float, L_int: int):
    """BranchSampler::gradient_descent (branch_sampler.rs:964-1002): L ascent steps
    theta += s * ldg (descend_gradient, params.rs:740-749), s from a doubling /
    halving line search over rss probes from the step size factor
    (probe_gradient_step, 1004-1016); always accepted.  ``br`` moves in place."""
    th = param_vec(br.weights, br.biases)

    def set_th(v):
        br.weights, br.biases = load_param_vec(v, br.num_markers, br.layer_widths)

    def grad():
        gw, gb, _ = log_density_gradient(br, X, y)
        return param_vec(gw, gb)

    def probe(step):
        set_th(th + step * g)
        return rss(br, X, y)

    g = grad()
    for _ in range(L_int):
        step = float(np.float32(factor))
        prev = probe(step)
        f = 2.0 if probe(2.0 * step) < prev else 0.5
        step *= f
        curr = probe(step)
        guard = 0
        while curr < prev and guard < 4096:
            prev = curr
            step *= f
            curr = probe(step)
            guard += 1
        step /= f
        th = th + step * g
        set_th(th)
        g = grad()
    set_th(th)
    return dict(status=ACCEPTED)


def gradient_descent_joint(br: Branch, X, y, hp: "Hyper", factor: float, L_int: int):
    """BranchSampler::gradient_descent_joint (branch_sampler.rs:1019-1066): L steps
    of params and precisions along the joint log-density gradient at the fixed
    factor; rejected (restored) if the error precision ends <= 0."""
    P = br.num_params
    init = br.copy()
    g, _ = ldg_joint_vec(br, X, y, hp)
    for _ in range(L_int):
        v = np.concatenate([param_vec(br.weights, br.biases), precision_vec(br)]) + float(np.float32(factor)) * g
        br.weights, br.biases = load_param_vec(v[:P], br.num_markers, br.layer_widths)
        load_precision_vec(br, v[P:])
        with np.errstate(all="ignore"):
            g, _ = ldg_joint_vec(br, X, y, hp)
    if not (br.error_precision > 0.0):
        br.weights, br.biases = init.weights, init.biases
        load_precision_vec(br, precision_vec(init))
        return dict(status=REJECTED)
    return dict(status=ACCEPTED)


# --------------------------------------------------------------------------
# network-joint HMC (bann_network_hmc_step; SURVEY 8(e) packed-joint mode)
# --------------------------------------------------------------------------
def network_hmc_step(brs: Sequence[Branch], Xs, y, bias: float, lambda_e: float, eps_list, p_list, L_int: int,
                     max_dH: float, u: float):
    """One HMC state over the parameters of every branch:
        -U = -lambda_e/2 ||sum_b f_b + bias - y||^2 + sum_b log prior_b
    (log prior_b = log_density(b, rss = 0): the branch's own prior terms,
    branch_sampler.rs:72-78 / std_normal_branch.rs:149-158).  The gradient of
    branch b is its backpropagate (813-875) against the target f_b - e, e the
    network error, i.e. J_b^T e.  Leapfrog as hmc_step (1239-1262), one
    Metropolis decision for the network; a divergence at any step rejects
    early.  eps_list / p_list: per-branch param_vec-ordered vectors.  Branches
    are updated in place (restored on rejection)."""
    brs = list(brs)
    for b in brs:
        b.error_precision = lambda_e
    init = [b.copy() for b in brs]
    eps = [np.asarray(e, dtype=np.float64) for e in eps_list]
    p = [np.array(x, dtype=np.float64) for x in p_list]

    def grads():
        preds = [predict(b, X) for b, X in zip(brs, Xs)]
        e = sum(preds) + bias - y
        gs = []
        for b, X, f in zip(brs, Xs, preds):
            gw, gb, _ = log_density_gradient(b, X, f - e)
            gs.append(param_vec(gw, gb))
        return gs, float(e @ e)

    def neg_h(rss_v):
        return (sum(log_density(b, 0.0) for b in brs) - lambda_e * rss_v / 2.0
                - 0.5 * sum(float(q @ q) for q in p))

    g, r = grads()
    H0 = neg_h(r)
    trace = [H0]
    status = ACCEPTED
    for step in range(L_int):
        for k, b in enumerate(brs):
            p[k] += 0.5 * eps[k] * g[k]
            th = param_vec(b.weights, b.biases) + eps[k] * p[k]
            b.weights, b.biases = load_param_vec(th, b.num_markers, b.layer_widths)
        g, r = grads()
        for k in range(len(brs)):
            p[k] += 0.5 * eps[k] * g[k]
        H = neg_h(r)
        trace.append(H)
        if abs(H - H0) > max_dH:
            status = REJECTED_EARLY
            break
    if status == ACCEPTED:
        log_acc = trace[-1] - H0
        acc_p = 1.0 if log_acc >= 0 else math.exp(log_acc)
        status = ACCEPTED if u < acc_p else REJECTED
    if status != ACCEPTED:
        for b, b0 in zip(brs, init):
            b.weights, b.biases = b0.weights, b0.biases
    return dict(status=status, trace=trace, rss=r)


def common_mode_gains(brs: Sequence[Branch], Xs):
    """g_b = J_b^T 1 per branch (param_vec order): the gradient of sum_i f_b(i), i.e. the
    half-rss backward (branch_sampler.rs:813-875) against the target f_b - 1."""
    gs = []
    for b, X in zip(brs, Xs):
        f = predict(b, X)
        _, dW, db = backpropagate(b, X, f - 1.0)
        gs.append(param_vec(dW, db))
    return gs


def common_mode_steps(brs: Sequence[Branch], Xs, eps_list, lambda_e: float, tau: float = 1.0):
    """The network-joint step-size rule (bann_set_network_step_rule; no reference counterpart,
    DESIGN.md 7), exact water-filling in f64: with a_p = eps_p |g_p| (g = J^T 1 over every
    branch), eps_p min(1, t / a_p) with the largest t such that lambda_e / n sum_p min(a_p, t)^2
    <= tau^2 (t = inf when the unscaled sum already is).  Returns (new eps list, t, a list)."""
    n = Xs[0].shape[0]
    gs = common_mode_gains(brs, Xs)
    a = [np.asarray(e, np.float64) * np.abs(g) for e, g in zip(eps_list, gs)]
    allv = np.sort(np.concatenate(a))[::-1]
    T = tau * tau * n / lambda_e
    if float(np.sum(allv * allv)) <= T:
        return [np.asarray(e, np.float64).copy() for e in eps_list], math.inf, a
    # f(t) = k t^2 + sum_{p >= k} a_(p)^2 with the k largest capped: find the crossing
    tail = np.concatenate([np.cumsum((allv * allv)[::-1])[::-1], [0.0]])
    t = 0.0
    for k in range(1, allv.size + 1):
        # t in [a_(k), a_(k-1)] with k capped: k t^2 + tail[k] = T
        tk2 = (T - tail[k]) / k
        lo = allv[k] if k < allv.size else 0.0
        if tk2 >= lo * lo:
            t = math.sqrt(max(tk2, 0.0))
            break
    return [np.asarray(e, np.float64) * np.minimum(1.0, t / np.maximum(x, 1e-300)) for e, x in zip(eps_list, a)], t, a


# --------------------------------------------------------------------------
# Gibbs precision posteriors (host side): gibbs_steps.rs, ridge_ard.rs:271-301
# --------------------------------------------------------------------------
def ridge_posterior_params(shape: float, scale: float, sum_sq: float, num: int):
    """gibbs_steps.rs:76-94 / 113-129: Gamma(shape + num/2, 2s / (2 + s * sum_sq))."""
    return shape + num / 2.0, 2.0 * scale / (2.0 + scale * sum_sq)


def lasso_posterior_params(shape: float, scale: float, sum_abs: float, num: int):
    """gibbs_steps.rs:25-57: Gamma(shape + num, s / (1 + s * sum_abs))."""
    return shape + num, scale / (1.0 + scale * sum_abs)


def ard_row_posterior_params(br: Branch, l: int, hp: Hyper):
    """ridge_ard.rs:271-291 / lasso_ard.rs:271-292: per-input-node Gamma posteriors."""
    shape, scale = hp.layer(l, br.num_layers)
    w = br.weights[l]
    width = br.layer_widths[l]
    if br.prior == "ridge_ard":
        return [(width / 2.0 + shape, 2.0 * scale / (2.0 + scale * s)) for s in _row_sumsq(w)]
    return [(width + shape, scale / (1.0 + scale * s)) for s in _row_l1(w)]


# --------------------------------------------------------------------------
# PLINK .bed codec: src/io/bed.rs:193-245, 325-355, bed_lookup_tables.rs:4
# --------------------------------------------------------------------------
# 2-bit code -> genotype (LUT of bed_lookup_tables.rs:4): 00->2, 01->0 (missing), 10->1, 11->0
BED_CODE_TO_GENOTYPE = np.array([2, 0, 1, 0], dtype=np.int8)


def bed_decode(data: bytes, n: int, m: int) -> np.ndarray:
    """Variant-major .bed payload (signature stripped) -> int8 genotypes [m][n].

    bed.rs:272-289 (get_cols) / 325-355.
    """
    bpc = (n + 3) // 4
    raw = np.frombuffer(bytes(data), dtype=np.uint8)[: bpc * m].reshape(m, bpc)
    codes = np.stack([(raw >> (2 * k)) & 3 for k in range(4)], axis=-1).reshape(m, bpc * 4)
    return BED_CODE_TO_GENOTYPE[codes[:, :n]]


def bed_col_stats_f32(g: np.ndarray):
    """bed.rs:231-242: f32 mean and population std, sequential f32 sums (exact
    reference rounding; use on small fixtures only)."""
    m, n = g.shape
    means = np.zeros(m, dtype=np.float32)
    stds = np.zeros(m, dtype=np.float32)
    nf = np.float32(n)
    for j in range(m):
        s = np.float32(0)
        for v in g[j]:
            s = np.float32(s + np.float32(v))
        mean = np.float32(s / nf)
        q = np.float32(0)
        for v in g[j]:
            d = np.float32(np.float32(v) - mean)
            q = np.float32(q + d * d)
        means[j] = mean
        stds[j] = np.float32(np.sqrt(np.float32(q / nf)))
    return means, stds


def bed_col_stats(g: np.ndarray):
    """float64 column mean / population std (bed.rs:231-242 semantics)."""
    gf = g.astype(np.float64)
    mu = gf.mean(axis=1)
    sd = np.sqrt(((gf - mu[:, None]) ** 2).mean(axis=1))
    return mu, sd


def standardized_submatrix(g: np.ndarray, mu, sd, cols, dtype=np.float32) -> np.ndarray:
    """bed.rs:325-355: (g - mu) / sd for the selected columns, (n x len(cols))."""
    cols = np.asarray(cols, dtype=np.int64)
    x = g[cols].T.astype(dtype)
    return ((x - np.asarray(mu, dtype=dtype)[cols][None, :]) / np.asarray(sd, dtype=dtype)[cols][None, :]).astype(dtype)


def bed_encode(g: np.ndarray) -> bytes:
    """Inverse of bed_decode (bed.rs vecf32_to_bed semantics): genotype -> 2-bit code."""
    m, n = g.shape
    code = {0: 3, 1: 2, 2: 0}
    bpc = (n + 3) // 4
    out = np.zeros((m, bpc), dtype=np.uint8)
    c = np.vectorize(code.get)(g).astype(np.uint8)
    pad = np.full((m, bpc * 4 - n), 0, dtype=np.uint8)
    c = np.concatenate([c, pad], axis=1).reshape(m, bpc, 4)
    for k in range(4):
        out |= (c[:, :, k] << (2 * k)).astype(np.uint8)
    return out.tobytes()


# --------------------------------------------------------------------------
# builders used by tests / bench
# --------------------------------------------------------------------------
def kat_branch(prior: str = "ridge_ard", precision: float = 1.0) -> Branch:
    """The tiny branch of every hot-path KAT (ridge_ard.rs:355-408; BranchBuilder
    branch_builder.rs:444-535).  widths [2,1,1], m=3, all precisions equal."""
    weights = [np.array([0.0, 1, 2, 3, 4, 5]).reshape((3, 2), order="F"),
               np.array([[1.0], [2.0]]), np.array([[2.0]])]
    biases = [np.array([0.0, 1.0]), np.array([2.0])]
    L = 3
    if prior in ARD_PRIORS:
        wp = [np.full(3, precision), np.full(2, precision), np.full(1, precision)]
    else:
        wp = [np.full(1, precision) for _ in range(L)]
    return Branch(3, [2, 1, 1], prior, "tanh", weights, biases, wp, [precision] * (L - 1), precision,
                  out_reg_sum=0.0, out_num_params=1.0)


def kat_data():
    """X (4x3, column-major) and y of the KATs (ridge_ard.rs:457-460, 529)."""
    X = np.array([1.0, 0, 0, 2, 1, 1, 2, 0, 0, 2, 0, 1]).reshape((4, 3), order="F")
    y = np.array([0.0, 2.0, 1.0, 1.5])
    return X, y


def random_branch(rng: np.random.Generator, m: int, widths: Sequence[int], prior="ridge_ard",
                  act="tanh", error_precision=2.0) -> Branch:
    """Default init (branch_cfg_builder.rs:180-186): W ~ N(0, 1/m), biases 0 (here
    small random biases so the bias gradients are exercised), ARD ML precisions
    (branch_cfg_builder.rs:308-328), base ML precisions (240-262)."""
    widths = list(widths)
    ins = [m] + widths[:-1]
    weights = [rng.normal(0.0, math.sqrt(1.0 / m), size=(i, o)) for i, o in zip(ins, widths)]
    biases = [rng.normal(0.0, 0.1, size=o) for o in widths[:-1]]
    L = len(widths)
    wp = []
    for l in range(L):
        w = weights[l]
        if prior in ARD_PRIORS and l < L - 1:
            wp.append(widths[l] / np.sum(w * w, axis=1))
        else:
            wp.append(np.array([w.size / np.sum(w * w)]))
    bp = [float(b.size / np.sum(b * b)) for b in biases]
    return Branch(m, widths, prior, act, weights, biases, wp, bp, error_precision,
                  out_reg_sum=0.0, out_num_params=float(weights[-1].size))


def synthetic_genotypes(rng: np.random.Generator, n: int, m: int) -> np.ndarray:
    """g_ij ~ Binomial(2, p_j), p_j ~ U(0.01, 0.5), zero-variance columns
    redrawn (bed.rs:136-188 semantics, numpy PCG64 stream).  Returns int8 [m][n]."""
    g = np.empty((m, n), dtype=np.int8)
    for j in range(m):
        while True:
            p = rng.uniform(0.01, 0.5)
            col = rng.binomial(2, p, size=n).astype(np.int8)
            if n == 1 or col.min() != col.max():
                g[j] = col
                break
    return g
