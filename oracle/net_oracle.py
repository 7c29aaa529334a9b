"""CPU oracle of the sequential network driver and the Net<B> model file.

TEST INFRASTRUCTURE ONLY (same rule as bann_oracle.py): only ``tests/`` may
import this module, as the checker of librsbann_amd.so's bann_net_* entry
points (include/bann_net.h).

* ``NetOracle.train`` restates ``Net::train`` (medical-genomics-group/rs-bann
  src/net/net.rs:201-358) for the HMC path, float64, on the per-branch oracle
  math of bann_oracle.py.  Random draws come from a ``Draws`` stream in the
  order documented in include/bann_net.h, so a device run whose RNG hooks
  replay the same stream takes the same decisions (the reference's ThreadRng
  is unseeded: the stream itself is parity-unpinned, the arithmetic is not).
* ``read_net_file`` parses the bincode 1.3 (legacy: fixint, little-endian)
  encoding of the ``Net<B>`` struct field by field.  No
  reference model file ships with the reference, so the layout is pinned by the
  struct declarations it follows (cited per field), not by a fixture.
"""
from __future__ import annotations

import math
import struct
from typing import List

import numpy as np

import bann_oracle as O


class Draws:
    """the shared random stream (numpy PCG64)."""

    def __init__(self, seed: int):
        self.rng = np.random.default_rng(seed)

    def uniform(self) -> float:
        return float(self.rng.random())

    def normal(self) -> float:
        return float(self.rng.standard_normal())

    def gamma(self, shape: float, scale: float) -> float:
        return float(self.rng.gamma(shape, scale))


def out_stat(br: O.Branch) -> float:
    """summary_stat_fn_host of the output weights (ridge_ard.rs:39-41, lasso_ard.rs:45-47)."""
    w = br.weights[-1]
    return float(np.sum(np.abs(w))) if br.prior.startswith("lasso") else float(np.sum(w * w))


class NetOracle:
    """Net<B> over oracle branches; X[b] = the standardized n x m_b block of branch b."""

    def __init__(self, branches: List[O.Branch], X: List[np.ndarray], hp: O.Hyper):
        self.br = [b.copy() for b in branches]
        self.X = X
        self.hp = hp
        nb = len(branches)
        # BlockNetCfg::build_net (architectures.rs:187-237)
        self.g_eprec = 2.0
        self.g_oprec = float(np.asarray(branches[0].weight_precisions[-1]).reshape(-1)[0])
        self.g_reg = sum(out_stat(b) for b in self.br)
        self.g_num = float(sum(b.weights[-1].size for b in self.br))
        self.ob_eprec, self.ob_prec, self.ob_bias = 2.0, 1.0, 0.0   # OutputBias (architectures.rs:224-228)
        self.ns = self.nacc = self.nearly = 0                           # TrainingStats
        self.mse, self.lpd = [], []
        self.lpd_rss = self.lpd_outw = -math.inf                         # LogPosteriorDensity
        self.lpd_local = [-math.inf] * nb
        self.residual = None

    # BranchCfg::update_global_params (branch_cfg.rs:59-63) + from_cfg (branch_struct.rs:26)
    def _from_cfg(self, b: int) -> float:
        br = self.br[b]
        br.error_precision = self.g_eprec
        br.weight_precisions[-1] = np.array([self.g_oprec])
        others = self.g_reg - out_stat(br)
        br.out_reg_sum, br.out_num_params = others, self.g_num
        return others

    def _update_lpd(self, b: int):
        """LogPosteriorDensity::update_from_branch (log_posterior_density.rs:27-61)"""
        br = self.br[b]
        self.lpd_local[b] = O.ld_joint_wrt_local_weights(br, self.hp) + O.ld_joint_wrt_biases(br, self.hp)
        self.lpd_outw = O.ld_joint_wrt_output_weights(br, self.hp)
        k, s = self.hp.output
        rss = float(np.sum(self.residual ** 2))
        le = br.error_precision
        self.lpd_rss = math.log(le) * (k + (self.residual.size - 2.0) / 2.0) - le * (rss / 2.0 + 1.0 / s)

    def _record(self):
        """Net::record_perf (net.rs:597-610)"""
        self.lpd.append(self.lpd_rss + self.lpd_outw + sum(self.lpd_local))
        self.mse.append(float(np.sum(self.residual ** 2)) / self.residual.size)

    def _sample_prior_precisions(self, br: O.Branch, d: Draws):
        """ridge_ard.rs:271-301, lasso_ard.rs:271-298, ridge_base.rs / lasso_base.rs"""
        L = br.num_layers
        for l in range(L - 1):
            shape, scale = self.hp.layer(l, L)
            w = br.weights[l]
            if br.prior in O.ARD_PRIORS:
                br.weight_precisions[l] = np.array([d.gamma(a, s) for a, s in O.ard_row_posterior_params(br, l, self.hp)])
            elif br.prior == "lasso_base":
                a, s = O.lasso_posterior_params(shape, scale, float(np.sum(np.abs(w))), w.size)
                br.weight_precisions[l] = np.array([d.gamma(a, s)])
            else:
                a, s = O.ridge_posterior_params(shape, scale, float(np.sum(w * w)), w.size)
                br.weight_precisions[l] = np.array([d.gamma(a, s)])
            bb = br.biases[l]
            a, s = O.ridge_posterior_params(shape, scale, float(np.sum(bb * bb)), bb.size)
            br.bias_precisions[l] = d.gamma(a, s)

    def train(self, y, d: Draws, chain_length: int, L_int: int, max_dH: float = 10.0, factor: float = 1.0,
              step_mode: str = "izmailov", fixed_param_precisions: bool = False, sampled_output_bias: bool = False,
              joint_hmc: bool = False, single_branch: bool = False, gradient_descent: bool = False,
              gradient_descent_joint: bool = False):
        """Net::train (net.rs:201-358); single_branch: Net::train_single_branch
        (net.rs:360-507: branch 0 every chain iteration, a record after every update).
        The step (282-290): gradient descent, joint gradient descent, joint HMC, HMC."""
        n = y.size
        nb = len(self.br)
        k_out, s_out = self.hp.output
        # initialize_stats (158-171)
        self.residual = np.asarray(y, dtype=np.float64) - self.ob_bias
        for b in range(nb):
            self._from_cfg(b)
            self.residual = self.residual - O.predict(self.br[b], self.X[b])
            self._update_lpd(b)
        self._record()
        order = list(range(nb))
        for _chain in range(chain_length):
            if single_branch:
                order = [0]
            else:
                for i in range(nb - 1, 0, -1):   # branch_ixs.shuffle (257)
                    j = min(i, int(math.floor(d.uniform() * (i + 1))))
                    order[i], order[j] = order[j], order[i]
            for b in order:
                br = self.br[b]
                others = self._from_cfg(b)
                if not (joint_hmc or gradient_descent_joint):   # 270-277
                    # sample_error_precision (branch_sampler.rs:190-202)
                    a, s = O.ridge_posterior_params(k_out, s_out, float(np.sum(self.residual ** 2)), n)
                    br.error_precision = d.gamma(a, s)
                    if not fixed_param_precisions:   # sample_param_precisions (173-188)
                        self._sample_prior_precisions(br, d)
                        total = others + out_stat(br)
                        post = O.lasso_posterior_params if br.prior.startswith("lasso") else O.ridge_posterior_params
                        a, s = post(k_out, s_out, total, self.g_num)
                        br.weight_precisions[-1] = np.array([d.gamma(a, s)])
                prev = O.predict(br, self.X[b])                                   # 279-280
                self.residual = self.residual + prev
                target = self.residual.astype(np.float32).astype(np.float64)      # the f32 target on the device
                f32 = lambda v: np.float64(np.float32(v))   # noqa: E731  (the device's f32 draws)
                if gradient_descent:   # branch_sampler.rs:964-1016
                    out = O.gradient_descent(br, self.X[b], target, factor, L_int)
                elif gradient_descent_joint:   # 1019-1066
                    br.out_reg_sum, br.out_num_params = others, self.g_num
                    out = O.gradient_descent_joint(br, self.X[b], target, self.hp, factor, L_int)
                elif joint_hmc:   # hmc_step_joint (branch_sampler.rs:1070-1178), random step sizes (654-704)
                    P, Q = br.num_params, O.precision_vec(br).size
                    f = np.float32(np.float32(P + Q) ** np.float32(-0.25)) * np.float32(factor)
                    eps = np.array([f32(np.float32(d.uniform()) * f) for _ in range(P + Q)])
                    p = np.array([f32(d.normal()) for _ in range(P + Q)])
                    u = f32(d.uniform())
                    out = O.hmc_step_joint(br, self.X[b], target, self.hp, eps, p, L_int, max_dH, u)
                else:
                    if step_mode == "random":   # random_step_sizes (654-681): drawn before the momentum
                        f = np.float32(np.float32(br.num_params) ** np.float32(-0.25)) * np.float32(factor)
                        ev = np.array([f32(np.float32(d.uniform()) * f) for _ in range(br.num_params)])
                        ew, eb = O.load_param_vec(ev, br.num_markers, br.layer_widths)
                    p = np.array([d.normal() for _ in range(br.num_params)])
                    u = f32(d.uniform())
                    p_w, p_b = O.load_param_vec(p.astype(np.float32).astype(np.float64), br.num_markers,
                                                br.layer_widths)
                    if step_mode == "izmailov":
                        ew, eb = O.izmailov_step_sizes(br, factor, L_int)
                    elif step_mode == "uniform":
                        ew, eb = O.uniform_step_sizes(br, factor)
                    elif step_mode == "std_scaled":   # branch_sampler.rs:1213, ridge_base.rs:52-82
                        ew, eb = O.std_scaled_step_sizes(br, factor)
                        ew = [np.asarray(e, np.float64) for e in ew]
                        eb = [np.asarray(e, np.float64) for e in eb]
                    out = O.hmc_step(br, self.X[b], target, ew, eb, p_w, p_b, L_int, max_dH, u)
                self.ns += 1
                self.nacc += out["status"] == O.ACCEPTED
                self.nearly += out["status"] == O.REJECTED_EARLY
                if out["status"] == O.ACCEPTED:                                    # 292-300
                    self.residual = self.residual - O.predict(br, self.X[b])
                    self._update_lpd(b)
                else:
                    self.residual = self.residual - prev
                # to_cfg + GlobalParams::update_from_branch_cfg (303-305, params.rs:41-56)
                self.g_eprec = br.error_precision
                self.g_oprec = float(np.asarray(br.weight_precisions[-1]).reshape(-1)[0])
                self.g_reg = others + out_stat(br)
                # output bias (319-332)
                self.ob_eprec = self.g_eprec
                self.residual = self.residual + self.ob_bias
                sr = float(np.sum(self.residual))
                if sampled_output_bias:
                    # quirk: the prior SHAPE passed as the scale (net.rs:61-66)
                    self.ob_prec = d.gamma(k_out + 0.5, 2.0 * k_out / (2.0 + k_out * self.ob_bias ** 2))
                    den = n * self.ob_eprec + self.ob_prec
                    self.ob_bias = self.ob_eprec / den * sr + math.sqrt(1.0 / den) * d.normal()
                else:
                    self.ob_bias = sr / n
                self.residual = self.residual - self.ob_bias
                if single_branch:
                    self._record()
            if not single_branch:
                self._record()


# ------------------------------------------------------------------ model file
class _Rd:
    def __init__(self, data: bytes):
        self.d, self.p = data, 0

    def take(self, fmt):
        v = struct.unpack_from("<" + fmt, self.d, self.p)
        self.p += struct.calcsize("<" + fmt)
        return v[0] if len(v) == 1 else v

    def vec(self, fmt):
        k = self.take("Q")
        return [self.take(fmt) for _ in range(k)]


def read_net_file(path: str) -> dict:
    """bincode Net<B> (net.rs:74-85) -> nested dict, field names of the reference structs."""
    r = _Rd(open(path, "rb").read())
    hp = {k: {"shape": r.take("f"), "scale": r.take("f")} for k in ("dense", "summary", "output")}  # params.rs:134-142
    net = {"hyperparams": hp, "num_branches": r.take("Q"), "branch_cfgs": []}
    for _ in range(r.take("Q")):
        cfg = {"num_params": r.take("Q"), "num_weights": r.take("Q"), "num_markers": r.take("Q"),
               "layer_widths": r.vec("Q")}                                               # branch_cfg.rs:8-16
        cfg["params"] = {"weights": [r.vec("f") for _ in range(r.take("Q"))],             # params.rs:468-476
                         "biases": [r.vec("f") for _ in range(r.take("Q"))],
                         "layer_widths": r.vec("Q"), "num_markers": r.take("Q"),
                         "output_weight_summary_stats": {"reg_sum": r.take("f"), "num_params": r.take("Q")}}
        cfg["precisions"] = {"weight_precisions": [r.vec("f") for _ in range(r.take("Q"))],  # params.rs:192-199
                             "bias_precisions": [r.vec("f") for _ in range(r.take("Q"))],
                             "error_precision": r.vec("f")}
        cfg["activation_function"] = r.take("I")                                          # activation_functions.rs:6-12
        net["branch_cfgs"].append(cfg)
    net["output_bias"] = {"error_precision": r.take("f"), "precision": r.take("f"), "bias": r.take("f")}  # net.rs:29-36
    ts = {"num_samples": r.take("Q"), "num_accepted": r.take("Q"), "num_early_rejected": r.take("Q"),
          "mse_train": r.vec("f")}                                                        # train_stats.rs:24-32
    ts["mse_test"] = r.vec("f") if r.take("B") else None
    ts["lpd"] = r.vec("f")
    net["training_stats"] = ts
    net["log_posterior_density"] = {"wrt_rss_and_error_precision": r.take("f"),          # log_posterior_density.rs:9-16
                                    "wrt_output_weights_and_precision": r.take("f"),
                                    "wrt_local_params": r.vec("f")}
    net["global_params"] = {"error_precision": r.take("f"), "output_layer_precision": r.take("f"),  # params.rs:13-18
                            "output_weight_summary_stats": {"reg_sum": r.take("f"), "num_params": r.take("Q")}}
    assert r.p == len(r.d), f"{len(r.d) - r.p} trailing bytes"                            # PhantomData: 0 bytes
    return net
