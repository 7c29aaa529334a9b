"""Host mirror of include/bann_net.h: the sequential network driver.

``Net`` wraps a ``bann_net`` over a finalized ``BannContext``: ``train`` is
``Net::train`` (src/net/net.rs:201-358) -- per sweep the branches in shuffled
order, each fitted by one HMC trajectory on the device against the residual
refreshed after the previous branch, Gibbs precision draws, the output bias and
the log posterior density on the host -- and ``save`` / ``load`` are
``Net::to_file`` / ``from_file`` (net.rs:107-115, bincode ``Net<B>``).  All
computation is in librsbann_amd.so (C++ driver + HIP kernels).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Callable, Optional, Tuple

import numpy as np

from ._lib import (GAMMA_FN, NORMAL_FN, STEP_MODES, UNIFORM_FN, BannError, McmcCfg, PrecisionHyperparams,
                   RngHooks, TrainSummary)

VAGUE = (0.001, 1000.0)  # PrecisionHyperparameters::vague (params.rs:119-124)


@dataclass
class MCMCConfig:
    """The MCMCCfg fields of Net::train's HMC path; defaults of MCMCCfgBuilder::default
    (mcmc_cfg.rs:34-56).  burn_in None -> chain_length - 1 (mcmc_cfg.rs:152-156)."""
    hmc_step_size_factor: float = 1.0
    hmc_max_hamiltonian_error: float = 10.0
    hmc_integration_length: int = 100
    hmc_step_size_mode: str = "izmailov"
    chain_length: int = 100
    burn_in: Optional[int] = None
    fixed_param_precisions: bool = False
    sampled_output_bias: bool = False
    trace: bool = False          # outdir/trace: BranchCfgs as JSON per sweep (net.rs:241-244, 350-353)
    trajectories: bool = False   # outdir/traj: one Trajectory JSON per HMC step (trajectory.rs)
    joint_hmc: bool = False      # hmc_step_joint over params and precisions, no Gibbs draws (net.rs:270-290)
    gradient_descent: bool = False        # BranchSampler::gradient_descent (line search, branch_sampler.rs:964-1016)
    gradient_descent_joint: bool = False  # gradient_descent_joint (params and precisions, 1019-1066)
    effect_sizes: bool = False   # outdir/effect_sizes/<chain_ix>_<branch_ix> CSVs after burn-in (net.rs:307-315)

    def to_c(self) -> McmcCfg:
        burn = self.chain_length - 1 if self.burn_in is None else self.burn_in
        return McmcCfg(self.hmc_step_size_factor, self.hmc_max_hamiltonian_error, self.hmc_integration_length,
                       STEP_MODES[self.hmc_step_size_mode], self.chain_length, max(burn, 0),
                       int(self.fixed_param_precisions), int(self.sampled_output_bias), int(self.trace),
                       int(self.trajectories), int(self.joint_hmc), int(self.gradient_descent),
                       int(self.gradient_descent_joint), int(self.effect_sizes))


class Net:
    """Net<B> over every branch of ``ctx`` (branch params / precisions = the
    initial BranchCfgs).  hyperparams: ((dense shape, scale), (summary ...),
    (output ...)) = NetworkPrecisionHyperparameters."""

    def __init__(self, ctx, hyperparams: Tuple = (VAGUE, VAGUE, VAGUE), seed: int = 0):
        self._ctx = ctx
        self._lib = ctx._lib
        (ds, dc), (ss, sc), (os_, oc) = hyperparams
        self.hyperparams = hyperparams
        hp = PrecisionHyperparams(ds, dc, ss, sc, os_, oc)
        h = C.c_void_p()
        rc = self._lib.bann_net_create(ctx._h, C.byref(hp), seed, C.byref(h))
        if rc != 0:
            raise BannError(rc, "bann_net_create failed (std-normal branches cannot be trained, net.rs:167)")
        self._h = h
        self._hooks = None

    def _check(self, rc):
        if rc < 0:
            raise BannError(rc, self._lib.bann_net_last_error(self._h).decode())
        return rc

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.bann_net_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_rng(self, uniform: Callable[[], float], normal: Callable[[], float],
                gamma: Callable[[float, float], float]):
        """replace the driver's host RNG (draw order: include/bann_net.h)."""
        self._hooks = RngHooks(None, UNIFORM_FN(lambda _u: uniform()), NORMAL_FN(lambda _u: normal()),
                               GAMMA_FN(lambda _u, k, s: gamma(k, s)))
        self._check(self._lib.bann_net_set_rng_hooks(self._h, C.byref(self._hooks)))

    def set_global(self, error_precision: float, output_layer_precision: float, output_bias: float = 0.0,
                   output_bias_precision: float = 1.0):
        self._check(self._lib.bann_net_set_global(self._h, error_precision, output_layer_precision, output_bias,
                                                  output_bias_precision))

    def train(self, y, cfg: MCMCConfig = MCMCConfig(), outdir: Optional[str] = None):
        v = np.ascontiguousarray(y, dtype=np.float32)
        self._check(self._lib.bann_net_train(self._h, v.ctypes.data_as(C.POINTER(C.c_float)), v.size,
                                             C.byref(cfg.to_c()), outdir.encode() if outdir else None))

    def train_single_branch(self, y, cfg: MCMCConfig = MCMCConfig(), outdir: Optional[str] = None):
        """Net::train_single_branch (net.rs:360-507): branch 0, one update per chain iteration."""
        v = np.ascontiguousarray(y, dtype=np.float32)
        self._check(self._lib.bann_net_train_single_branch(self._h, v.ctypes.data_as(C.POINTER(C.c_float)), v.size,
                                                           C.byref(cfg.to_c()), outdir.encode() if outdir else None))

    def perturb(self, params_by: Optional[float] = None, precisions_by: Optional[float] = None):
        """Net::perturb (net.rs:187-199): shift every param and / or precision by a constant."""
        self._check(self._lib.bann_net_perturb(self._h, int(params_by is not None), float(params_by or 0.0),
                                               int(precisions_by is not None), float(precisions_by or 0.0)))

    def predict(self, ctx=None) -> np.ndarray:
        """Net::predict (net.rs:545-559): bias + sum_b f_b on ctx's cohort (default: the training context)."""
        c = ctx if ctx is not None else self._ctx
        out = np.zeros(c.n, np.float32)
        self._check(self._lib.bann_net_predict(self._h, c._h if ctx is not None else None,
                                               out.ctypes.data_as(C.POINTER(C.c_float))))
        return out

    def _ctxh(self, ctx):
        return ctx._h if ctx is not None else None

    def rss(self, y, ctx=None) -> float:
        """Net::rss (net.rs:637-642): sum (y - predict)^2 on ctx's cohort (default: training)."""
        v = np.ascontiguousarray(y, dtype=np.float32)
        r = C.c_double()
        self._check(self._lib.bann_net_rss(self._h, self._ctxh(ctx), v.ctypes.data_as(C.POINTER(C.c_float)), v.size,
                                           C.byref(r)))
        return r.value

    def mse(self, y, ctx=None) -> float:
        """Net::mse (net.rs:644-646)."""
        return self.rss(y, ctx) / np.asarray(y).size

    def gradient(self, y, ctx=None):
        """Net::gradient (net.rs:520-527): per branch the log-density gradient against y (param_vec order)."""
        c = ctx if ctx is not None else self._ctx
        v = np.ascontiguousarray(y, dtype=np.float32)
        sizes = [c.num_params(b) for b in range(c.num_branches)]
        out = np.zeros(sum(sizes), np.float32)
        self._check(self._lib.bann_net_gradient(self._h, self._ctxh(ctx), v.ctypes.data_as(C.POINTER(C.c_float)),
                                                v.size, out.ctypes.data_as(C.POINTER(C.c_float))))
        return np.split(out, np.cumsum(sizes)[:-1])

    def branch_r2s(self, y, ctx=None) -> np.ndarray:
        """Net::branch_r2s (net.rs:648-656): 1 - rss_b / sum y^2 per branch."""
        c = ctx if ctx is not None else self._ctx
        v = np.ascontiguousarray(y, dtype=np.float32)
        out = np.zeros(c.num_branches, np.float32)
        self._check(self._lib.bann_net_branch_r2s(self._h, self._ctxh(ctx), v.ctypes.data_as(C.POINTER(C.c_float)),
                                                  v.size, out.ctypes.data_as(C.POINTER(C.c_float))))
        return out

    def activations(self, b: int, ctx=None):
        """Net::activations (net.rs:509-518) of branch b: per layer an [n, w_l] array."""
        c = ctx if ctx is not None else self._ctx
        _, L, widths, _, _ = c.branch_info(b)
        out = np.zeros(sum(widths) * c.n, np.float32)
        self._check(self._lib.bann_net_activations(self._h, self._ctxh(ctx), b,
                                                   out.ctypes.data_as(C.POINTER(C.c_float))))
        res, o = [], 0
        for w in widths:
            res.append(out[o: o + w * c.n].reshape(w, c.n).T)
            o += w * c.n
        return res

    def population_effect_sizes(self, ctx=None) -> np.ndarray:
        """Net::population_effect_sizes (net.rs:529-543): per branch (branch order) the mean over
        ctx's individuals of effect_sizes (branch_sampler.rs:784-811), concatenated."""
        c = ctx if ctx is not None else self._ctx
        out = np.zeros(sum(c.branch_info(b)[0] for b in range(c.num_branches)), np.float32)
        self._check(self._lib.bann_net_population_effect_sizes(self._h, self._ctxh(ctx),
                                                               out.ctypes.data_as(C.POINTER(C.c_float))))
        return out

    def summary(self) -> dict:
        s = TrainSummary()
        self._check(self._lib.bann_net_summary(self._h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in TrainSummary._fields_}

    def records(self):
        """(mse_train, lpd) series of TrainingStats (train_stats.rs:24-32)."""
        k = self.summary()["num_records"]
        mse = np.zeros(k, np.float32)
        lpd = np.zeros(k, np.float32)
        self._check(self._lib.bann_net_records(self._h, mse.ctypes.data_as(C.POINTER(C.c_float)),
                                               lpd.ctypes.data_as(C.POINTER(C.c_float)), k))
        return mse, lpd

    def set_test_data(self, test_ctx, y_test):
        """record_perf's test set (net.rs:597-610): a context over the test cohort with the
        same branches; None detaches."""
        if test_ctx is None:
            self._check(self._lib.bann_net_set_test_data(self._h, None, None, 0))
            self._test = None
            return
        y = np.ascontiguousarray(y_test, dtype=np.float32)
        self._test = (test_ctx, y)   # the context must outlive the net's use of it
        self._check(self._lib.bann_net_set_test_data(self._h, test_ctx._h, y.ctypes.data_as(C.POINTER(C.c_float)),
                                                     y.size))

    def records_test(self) -> np.ndarray:
        k = self._lib.bann_net_records_test(self._h, None, 0)
        out = np.zeros(max(k, 0), np.float32)
        self._check(self._lib.bann_net_records_test(self._h, out.ctypes.data_as(C.POINTER(C.c_float)), out.size))
        return out

    def residual(self) -> np.ndarray:
        out = np.zeros(self._ctx.n, np.float32)
        self._check(self._lib.bann_net_residual(self._h, out.ctypes.data_as(C.POINTER(C.c_float))))
        return out

    def save(self, path: str):
        self._check(self._lib.bann_net_save(self._h, path.encode()))

    def load(self, path: str):
        self._check(self._lib.bann_net_load(self._h, path.encode()))
