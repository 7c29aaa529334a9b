"""Pythonic host mirror of the C ABI (include/bann.h).

``BannContext`` owns one device context.  Method names follow the reference's
BranchSampler / BranchStruct vocabulary (src/net/branch/branch_sampler.rs):
``predict``, ``rss``, ``log_density_gradient``, ``log_density``,
``neg_hamiltonian``, ``hmc_step``.  Every call goes through the HIP library;
nothing here computes on the CPU.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from ._lib import ACTIVATIONS, PRIORS, STEP_MODES, BannError, load_library


def _ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


class BannContext:
    def __init__(self, device: int = 0):
        self._lib = load_library()
        h = C.c_void_p()
        rc = self._lib.bann_ctx_create(int(device), C.byref(h))
        if rc != 0:
            raise BannError(rc, f"bann_ctx_create(device={device}) failed (no HIP device?)")
        self._h = h
        self.n = 0
        self.num_markers = 0
        self._branches = []

    # ------------------------------------------------------------------ util
    def _check(self, rc):
        if rc < 0:
            raise BannError(rc, self._lib.bann_last_error(self._h).decode())
        return rc

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.bann_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------- genotypes
    def upload_genotypes(self, g: np.ndarray):
        """g: int8 [num_markers][n] variant-major (bed.rs layout)."""
        g = np.ascontiguousarray(g, dtype=np.int8)
        M, n = g.shape
        self._check(self._lib.bann_genotypes_upload(self._h, _ptr(g, C.c_int8), n, M))
        self.n, self.num_markers = n, M

    def upload_bed(self, payload: bytes, n: int, num_markers: int):
        """variant-major .bed payload, ceil(n/4) bytes per marker; a full .bed file's
        3-byte signature (0x6c 0x1b 0x01, bed.rs:100-116) is stripped."""
        data = bytes(payload)
        want = ((n + 3) // 4) * num_markers
        if len(data) == want + 3 and data[:3] == b"\x6c\x1b\x01":
            data = data[3:]
        if len(data) != want:
            raise ValueError(f".bed payload has {len(data)} bytes, n={n} x {num_markers} markers need {want}")
        buf = np.frombuffer(data, dtype=np.uint8).copy()
        self._check(self._lib.bann_genotypes_upload_bed(self._h, _ptr(buf, C.c_uint8), n, num_markers))
        self.n, self.num_markers = n, num_markers

    def load_bed(self, stem: str):
        """PLINK stem.bed (+ .dims or .fam/.bim) streamed into the device image (bed.rs:193-245)."""
        self._check(self._lib.bann_genotypes_load_bed(self._h, stem.encode()))
        from .io import bed_dims
        self.n, self.num_markers = bed_dims(stem)

    def synthetic_genotypes(self, n: int, num_markers: int, seed: int = 42):
        self._check(self._lib.bann_genotypes_synthetic(self._h, n, num_markers, seed))
        self.n, self.num_markers = n, num_markers

    def genotype_stats(self):
        mu = np.zeros(self.num_markers, np.float32)
        sd = np.zeros(self.num_markers, np.float32)
        self._check(self._lib.bann_genotypes_stats(self._h, _ptr(mu, C.c_float), _ptr(sd, C.c_float)))
        return mu, sd

    def set_genotype_stats(self, mu, sigma):
        m = _f32(mu)
        s = _f32(sigma)
        self._check(self._lib.bann_genotypes_set_stats(self._h, _ptr(m, C.c_float), _ptr(s, C.c_float)))

    def download_genotypes(self, snp_idx: Sequence[int]) -> np.ndarray:
        idx = np.ascontiguousarray(snp_idx, dtype=np.int32)
        out = np.zeros((idx.size, self.n), np.int8)
        self._check(self._lib.bann_genotypes_download(self._h, _ptr(idx, C.c_int32), idx.size, _ptr(out, C.c_int8)))
        return out

    # -------------------------------------------------------------- branches
    def add_branch(self, snp_idx: Sequence[int], layer_widths: Sequence[int], activation: str = "tanh",
                   prior: str = "ridge_ard") -> int:
        idx = np.ascontiguousarray(snp_idx, dtype=np.int32)
        w = np.ascontiguousarray(layer_widths, dtype=np.int32)
        b = self._check(self._lib.bann_branch_add(self._h, _ptr(idx, C.c_int32), idx.size, _ptr(w, C.c_int32), w.size,
                                                  ACTIVATIONS[activation], PRIORS[prior]))
        self._branches.append((idx.copy(), list(layer_widths), activation, prior))
        return b

    def set_fused_enabled(self, enabled: bool):
        self._check(self._lib.bann_set_fused_enabled(self._h, 1 if enabled else 0))

    def finalize(self, free_raw: bool = False):
        self._check(self._lib.bann_finalize(self._h, 1 if free_raw else 0))

    @property
    def num_branches(self) -> int:
        return self._check(self._lib.bann_num_branches(self._h))

    def num_params(self, b: int) -> int:
        return int(self._check(self._lib.bann_num_params(self._h, b)))

    def num_precisions(self, b: int) -> int:
        return int(self._check(self._lib.bann_num_precisions(self._h, b)))

    def kernel_path(self, b: int) -> str:
        """"fused" (fx: widths <= 4, m <= 512), "fused_large" (fxl: widths <= 4, m <= 4096),
        "wide" (wx: one hidden layer <= 32 x 32, m <= 128) or "layered" (gx: any shape, layered MFMA GEMMs)."""
        return {1: "fused", 2: "wide", 3: "fused_large"}.get(
            self._check(self._lib.bann_branch_kernel_path(self._h, b)), "layered")

    def set_hidden_gemm_bf16(self, enabled: bool):
        """wide kernel: hidden GEMMs on bf16 MFMA (reduced precision) instead of f32 MFMA."""
        self._check(self._lib.bann_set_hidden_gemm_bf16(self._h, 1 if enabled else 0))

    def fused_kernel_name(self) -> str:
        return self._lib.bann_fused_kernel_name().decode()

    @property
    def packed_genotype_bytes(self) -> int:
        return int(self._lib.bann_packed_genotype_bytes(self._h))

    def set_params(self, b: int, param_vec):
        v = _f32(param_vec)
        assert v.size == self.num_params(b), "param_vec size"
        self._check(self._lib.bann_branch_set_params(self._h, b, _ptr(v, C.c_float)))

    def get_params(self, b: int) -> np.ndarray:
        out = np.zeros(self.num_params(b), np.float32)
        self._check(self._lib.bann_branch_get_params(self._h, b, _ptr(out, C.c_float)))
        return out

    def set_precisions(self, b: int, precision_vec):
        v = _f32(precision_vec)
        assert v.size == self.num_precisions(b), "precision_vec size"
        self._check(self._lib.bann_branch_set_precisions(self._h, b, _ptr(v, C.c_float)))

    def get_precisions(self, b: int) -> np.ndarray:
        out = np.zeros(self.num_precisions(b), np.float32)
        self._check(self._lib.bann_branch_get_precisions(self._h, b, _ptr(out, C.c_float)))
        return out

    def set_target(self, b: int, y):
        v = _f32(y)
        assert v.size == self.n
        self._check(self._lib.bann_branch_set_target(self._h, b, _ptr(v, C.c_float)))

    def set_target_all(self, y):
        v = _f32(y)
        assert v.size == self.n
        self._check(self._lib.bann_set_target_all(self._h, _ptr(v, C.c_float)))

    # ------------------------------------------------------- branch sampler
    def predict(self, b: int) -> np.ndarray:
        out = np.zeros(self.n, np.float32)
        self._check(self._lib.bann_predict(self._h, b, _ptr(out, C.c_float)))
        return out

    def get_step_sizes(self, b: int) -> np.ndarray:
        out = np.zeros(self.num_params(b), np.float32)
        self._check(self._lib.bann_branch_get_step_sizes(self._h, b, _ptr(out, C.c_float)))
        return out

    def predict_many(self, branches) -> np.ndarray:
        """(len(branches), n) predictions from one packed launch."""
        bl = np.ascontiguousarray(branches, dtype=np.int32)
        out = np.zeros((bl.size, self.n), np.float32)
        self._check(self._lib.bann_predict_many(self._h, _ptr(bl, C.c_int32), bl.size, _ptr(out, C.c_float)))
        return out

    def rss(self, b: int) -> float:
        r = C.c_double()
        self._check(self._lib.bann_rss(self._h, b, C.byref(r)))
        return r.value

    def log_density_gradient(self, b: int):
        g = np.zeros(self.num_params(b), np.float32)
        r = C.c_double()
        self._check(self._lib.bann_log_density_gradient(self._h, b, _ptr(g, C.c_float), C.byref(r)))
        return g, r.value

    def log_density_gradient_many(self, branches):
        """(list of param_vec gradients, rss array) of several branches from one packed launch."""
        bl = np.ascontiguousarray(branches, dtype=np.int32)
        sizes = [self.num_params(int(b)) for b in bl]
        g = np.zeros(sum(sizes), np.float32)
        r = np.zeros(bl.size, np.float64)
        self._check(self._lib.bann_log_density_gradient_many(self._h, _ptr(bl, C.c_int32), bl.size, _ptr(g, C.c_float),
                                                             _ptr(r, C.c_double)))
        return np.split(g, np.cumsum(sizes)[:-1]), r

    def log_density_gradient_joint(self, b: int, hyper):
        """(grad [P + Q], rss, joint log density) at the current params and precisions."""
        hp = _f32(hyper)
        if hp.size != 6:
            raise ValueError("hyper needs 6 values")
        g = np.zeros(self.num_params(b) + self.num_precisions(b), np.float32)
        r, ld = C.c_double(), C.c_double()
        self._check(self._lib.bann_log_density_gradient_joint(self._h, b, _ptr(hp, C.c_float), _ptr(g, C.c_float),
                                                              C.byref(r), C.byref(ld)))
        return g, r.value, ld.value

    def forward_feed(self, b: int, pre: bool = True):
        """forward_feed (branch_sampler.rs:743-782): (pre-activations, activations) as lists of
        [n, w_l] arrays per layer (the output layer's activation last; no pre-activation for it)."""
        _, L, widths, _, _ = self.branch_info(b)
        n = self.n
        act = np.zeros(sum(widths) * n, np.float32)
        pr = np.zeros(sum(widths[:-1]) * n, np.float32) if pre else None
        self._check(self._lib.bann_forward_feed(self._h, b, _ptr(pr, C.c_float) if pre else None,
                                                _ptr(act, C.c_float)))
        def split(v, ws):
            out, o = [], 0
            for w in ws:
                out.append(v[o: o + w * n].reshape(w, n).T)
                o += w * n
            return out
        return (split(pr, widths[:-1]) if pre else None), split(act, widths)

    def effect_sizes(self, b: int) -> np.ndarray:
        """BranchSampler::effect_sizes (branch_sampler.rs:784-811): the [n, m] matrix
        out_i d out_i / d x_ij at the branch's current parameters (output-seeded chain, no abs)."""
        m = self.branch_info(b)[0]
        out = np.zeros(m * self.n, np.float32)
        self._check(self._lib.bann_effect_sizes(self._h, b, _ptr(out, C.c_float)))
        return out.reshape(m, self.n).T

    def population_effect_sizes(self, branches) -> np.ndarray:
        """the per-branch column means of effect_sizes (Net::population_effect_sizes,
        net.rs:529-543), concatenated in list order."""
        bl = np.ascontiguousarray(branches, dtype=np.int32)
        out = np.zeros(sum(self.branch_info(int(b))[0] for b in bl), np.float32)
        self._check(self._lib.bann_population_effect_sizes(self._h, _ptr(bl, C.c_int32), bl.size,
                                                           _ptr(out, C.c_float)))
        return out

    def branch_info(self, b: int):
        """(markers, num_layers, layer widths, activation code, prior code) of branch b."""
        m, L, act, pr = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32()
        w = np.zeros(64, np.int32)
        self._check(self._lib.bann_branch_info(self._h, b, C.byref(m), C.byref(L), _ptr(w, C.c_int32), 64,
                                               C.byref(act), C.byref(pr)))
        return m.value, L.value, [int(v) for v in w[: L.value]], act.value, pr.value

    def log_density(self, b: int, rss: float) -> float:
        out = C.c_double()
        self._check(self._lib.bann_log_density(self._h, b, float(rss), C.byref(out)))
        return out.value

    def neg_hamiltonian(self, b: int, momentum) -> float:
        p = _f32(momentum)
        if p.size != self.num_params(b):
            raise ValueError(f"momentum has {p.size} entries, branch {b} has {self.num_params(b)} parameters")
        out = C.c_double()
        self._check(self._lib.bann_neg_hamiltonian(self._h, b, _ptr(p, C.c_float), C.byref(out)))
        return out.value

    def _check_sizes(self, br, eps, momentum, u, extra=None):
        """the C side reads sum(P_b) (+ extra(b)) floats of eps / momentum and one uniform per branch"""
        tot = sum(self.num_params(int(b)) + (extra(int(b)) if extra else 0) for b in br)
        for name, a in (("eps", eps), ("momentum", momentum)):
            if a is not None and a.size != tot:
                raise ValueError(f"{name} has {a.size} entries, the branches need {tot}")
        if u is not None and u.size != br.size:
            raise ValueError(f"u has {u.size} entries, expected one per branch ({br.size})")

    def hmc_step(self, branches: Sequence[int], L: int, max_hamiltonian_error: float = 10.0,
                 step_mode: str = "izmailov", step_factor: float = 1.0, eps=None, momentum=None, seed: int = 0,
                 u=None):
        """One HMC trajectory per branch, all branches packed (branch_sampler.rs:1192-1299)."""
        br = np.ascontiguousarray(branches, dtype=np.int32)
        nb = br.size
        eps_a = _f32(eps) if eps is not None else None
        mom_a = _f32(momentum) if momentum is not None else None
        u_a = _f32(u) if u is not None else None
        self._check_sizes(br, eps_a, mom_a, u_a)
        status = np.zeros(nb, np.int32)
        trace = np.zeros((nb, L + 1), np.float64)
        uturn = np.zeros(nb, np.int32)
        ld = np.zeros(nb, np.float64)
        mode = STEP_MODES["injected"] if eps is not None else STEP_MODES[step_mode]
        nullf = C.POINTER(C.c_float)()
        self._check(self._lib.bann_hmc_step(
            self._h, _ptr(br, C.c_int32), nb, L, max_hamiltonian_error, mode, step_factor,
            _ptr(eps_a, C.c_float) if eps_a is not None else nullf,
            _ptr(mom_a, C.c_float) if mom_a is not None else nullf, seed,
            _ptr(u_a, C.c_float) if u_a is not None else nullf,
            _ptr(status, C.c_int32), _ptr(trace, C.c_double), _ptr(uturn, C.c_int32), _ptr(ld, C.c_double)))
        return dict(status=status, trace=trace, uturn=uturn, log_density=ld)

    def set_trajectory_recording(self, enabled: bool):
        self._check(self._lib.bann_set_trajectory_recording(self._h, 1 if enabled else 0))

    def get_trajectory(self, b: int):
        """last recorded trajectory of branch b: dict(params [steps, P], ldg [steps, P], hamiltonian [steps+1])."""
        steps = C.c_int32()
        self._check(self._lib.bann_branch_get_trajectory(self._h, b, 0, C.byref(steps), None, None, None))
        k, P = steps.value, self.num_params(b)
        pr = np.zeros((k, P), np.float32)
        lg = np.zeros((k, P), np.float32)
        h = np.zeros(k + 1, np.float64)
        self._check(self._lib.bann_branch_get_trajectory(self._h, b, k, C.byref(steps), _ptr(pr, C.c_float),
                                                         _ptr(lg, C.c_float), _ptr(h, C.c_double)))
        return dict(params=pr, ldg=lg, hamiltonian=h)

    def get_trajectory_joint(self, b: int):
        """last recorded joint trajectory of branch b: dict(params [steps, P], precisions [steps, Q],
        ldg [steps, P + Q], hamiltonian [steps+1])."""
        steps = C.c_int32()
        self._check(self._lib.bann_branch_get_trajectory_joint(self._h, b, 0, C.byref(steps), None, None, None, None))
        k, P, Q = steps.value, self.num_params(b), self.num_precisions(b)
        pr = np.zeros((k, P), np.float32)
        pq = np.zeros((k, Q), np.float32)
        lg = np.zeros((k, P + Q), np.float32)
        h = np.zeros(k + 1, np.float64)
        self._check(self._lib.bann_branch_get_trajectory_joint(self._h, b, k, C.byref(steps), _ptr(pr, C.c_float),
                                                               _ptr(pq, C.c_float), _ptr(lg, C.c_float),
                                                               _ptr(h, C.c_double)))
        return dict(params=pr, precisions=pq, ldg=lg, hamiltonian=h)

    def set_graph_replay(self, enabled: bool):
        """bann_hmc_step: replay each trajectory's launch sequence as one captured HIP graph."""
        self._check(self._lib.bann_set_graph_replay(self._h, 1 if enabled else 0))

    def set_output_stats(self, b: int, reg_sum_others: float, num_params: float):
        """OutputWeightSummaryStats of branch b for the joint density (params.rs:404-465)."""
        self._check(self._lib.bann_branch_set_output_stats(self._h, b, float(reg_sum_others), float(num_params)))

    def hmc_step_joint(self, branches: Sequence[int], L: int, hyper, max_hamiltonian_error: float = 10.0,
                       step_factor: float = 1.0, eps=None, momentum=None, seed: int = 0, u=None):
        """hmc_step_joint (branch_sampler.rs:1070-1178): parameters and precisions.
        hyper: (dense shape, scale, summary shape, scale, output shape, scale);
        eps / momentum: per branch [num_params | num_precisions] (or None)."""
        br = np.ascontiguousarray(branches, dtype=np.int32)
        nb = br.size
        eps_a = _f32(eps) if eps is not None else None
        mom_a = _f32(momentum) if momentum is not None else None
        u_a = _f32(u) if u is not None else None
        hp = _f32(hyper)
        if hp.size != 6:
            raise ValueError("hyper needs 6 values")
        self._check_sizes(br, eps_a, mom_a, u_a, extra=self.num_precisions)
        status = np.zeros(nb, np.int32)
        trace = np.zeros((nb, L + 1), np.float64)
        ld = np.zeros(nb, np.float64)
        mode = STEP_MODES["injected"] if eps is not None else STEP_MODES["random"]
        nullf = C.POINTER(C.c_float)()
        self._check(self._lib.bann_hmc_step_joint(
            self._h, _ptr(br, C.c_int32), nb, L, max_hamiltonian_error, mode, step_factor,
            _ptr(eps_a, C.c_float) if eps_a is not None else nullf,
            _ptr(mom_a, C.c_float) if mom_a is not None else nullf, seed,
            _ptr(u_a, C.c_float) if u_a is not None else nullf, _ptr(hp, C.c_float),
            _ptr(status, C.c_int32), _ptr(trace, C.c_double), _ptr(ld, C.c_double)))
        return dict(status=status, trace=trace, log_density=ld)

    # ------------------------------------------------------ multi-GPU
    def comm_init_rccl(self, unique_id: bytes, nranks: int, rank: int):
        """RCCL communicator (collective: every rank calls it with rank 0's id)."""
        buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        self._check(self._lib.bann_ctx_comm_init(self._h, buf, nranks, rank))

    def comm_callback(self, allreduce, nranks: int, rank: int):
        """caller all-reduce (bann.distributed.TorchAllreduce) instead of RCCL."""
        self._allreduce = allreduce   # the library keeps the function pointer
        self._check(self._lib.bann_ctx_comm_callback(self._h, allreduce.fn, None, nranks, rank))

    def comm_info(self) -> dict:
        """the context's communicator: kind ("none" / "rccl" / "callback"), ranks, rank and
        the rank count the backend itself reports (ncclCommCount for RCCL)."""
        k, nr, r, br = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32()
        self._check(self._lib.bann_comm_info(self._h, C.byref(k), C.byref(nr), C.byref(r), C.byref(br)))
        return dict(kind={0: "none", 1: "rccl", 2: "callback"}[k.value], nranks=nr.value, rank=r.value,
                    backend_ranks=br.value)

    def exchange_residual(self, residual) -> np.ndarray:
        """residual -= sum over ranks of the last session's residual change (collective)."""
        res = np.ascontiguousarray(residual, dtype=np.float32).copy()
        self._check(self._lib.bann_exchange_residual(self._h, _ptr(res, C.c_float)))
        return res

    def network_hmc_step(self, y, L: int, bias: float = 0.0, lambda_e: float = 1.0,
                         max_hamiltonian_error: float = 10.0, step_mode: str = "izmailov",
                         step_factor: float = 1.0, eps=None, momentum=None, seed: int = 0,
                         u: Optional[float] = None):
        """network-joint HMC trajectory over every branch of every rank (collective).
        eps / momentum: concatenated over this context's branches in branch order (or None);
        u: injected Metropolis uniform (parity runs) or None: drawn on rank 0 from seed and
        shared with every rank by the library."""
        ya = _f32(y)
        if ya.size != self.n:
            raise ValueError(f"y has {ya.size} entries, n = {self.n}")
        br = np.arange(self.num_branches, dtype=np.int32)
        eps_a = _f32(eps) if eps is not None else None
        mom_a = _f32(momentum) if momentum is not None else None
        self._check_sizes(br, eps_a, mom_a, None)
        mode = STEP_MODES["injected"] if eps is not None else STEP_MODES[step_mode]
        nullf = C.POINTER(C.c_float)()
        st = C.c_int32()
        tr = np.zeros(L + 1, np.float64)
        rss = C.c_double()
        self._check(self._lib.bann_network_hmc_step(
            self._h, _ptr(ya, C.c_float), bias, lambda_e, L, max_hamiltonian_error, mode, step_factor,
            _ptr(eps_a, C.c_float) if eps_a is not None else nullf,
            _ptr(mom_a, C.c_float) if mom_a is not None else nullf, seed,
            C.byref(C.c_float(u)) if u is not None else nullf, C.byref(st), _ptr(tr, C.c_double),
            C.byref(rss)))
        return dict(status=st.value, trace=tr, rss=rss.value)

    def set_network_step_rule(self, common_mode="auto", tau: float = 1.0):
        """the network-joint state's step sizes (bann_set_network_step_rule): the common-mode
        water-filling rule at omega eps <= tau.  "auto" / 3 (the library default): adapted on
        the first K trajectories (set_network_adapt_trajectories, K = 1), then frozen; "frozen"
        / 2: the last adapted factors (state-independent steps); "adaptive" / True / 1:
        re-adapted before every trajectory (state-dependent proposals: a diagnostic);
        "off" / False / 0: the per-branch steps as given."""
        names = {"auto": 3, "frozen": 2, "adaptive": 1, "off": 0, True: 1, False: 0}
        mode = names[common_mode] if isinstance(common_mode, (str, bool)) else int(common_mode)
        self._check(self._lib.bann_set_network_step_rule(self._h, mode, float(tau)))

    def set_network_adapt_trajectories(self, k: int):
        """auto mode: the number of adapting trajectories before the factors freeze (restarts)."""
        self._check(self._lib.bann_set_network_adapt_trajectories(self._h, int(k)))

    def network_step_rule_state(self) -> dict:
        """mode, adapting trajectories done (auto mode), and whether the next trajectory
        applies frozen factors."""
        m, a, f = C.c_int32(), C.c_int32(), C.c_int32()
        self._check(self._lib.bann_network_step_rule_state(self._h, C.byref(m), C.byref(a), C.byref(f)))
        return dict(mode={0: "off", 1: "adaptive", 2: "frozen", 3: "auto"}[m.value], adapted=a.value,
                    frozen=bool(f.value))

    def network_group_rows(self) -> int:
        """the network forward's group-sum rows (k_forward_gsum), 0: per-branch rows, -1: not run yet"""
        r = C.c_int32()
        self._check(self._lib.bann_network_info(self._h, C.byref(r)))
        return r.value

    def network_step_rule_info(self) -> dict:
        """the last network trajectory's rule: threshold t, (omega eps)^2 of the common mode
        before and after, the fraction of parameters whose step was reduced."""
        out = np.zeros(4, np.float64)
        self._check(self._lib.bann_network_step_rule_info(self._h, _ptr(out, C.c_double)))
        return dict(threshold=out[0], mode_before=out[1], mode_after=out[2], fraction_scaled=out[3])

    def exchange_residual_device(self):
        """device residual -= sum over ranks of the last session's residual change (collective)."""
        self._check(self._lib.bann_exchange_residual_device(self._h))

    # ------------------------------------------------ device residual (net.rs:158-332)
    def residual_set(self, r):
        v = _f32(r)
        assert v.size == self.n
        self._check(self._lib.bann_residual_set(self._h, _ptr(v, C.c_float)))

    def residual_get(self) -> np.ndarray:
        out = np.zeros(self.n, np.float32)
        self._check(self._lib.bann_residual_get(self._h, _ptr(out, C.c_float)))
        return out

    def residual_init(self, y, bias: float = 0.0):
        """residual = (y - bias) - sum_b f_b (initialize_stats); returns (sum, sum of squares)."""
        v = _f32(y)
        s, q = C.c_double(), C.c_double()
        self._check(self._lib.bann_residual_init(self._h, _ptr(v, C.c_float), float(bias), C.byref(s), C.byref(q)))
        return s.value, q.value

    def residual_stats(self):
        s, q = C.c_double(), C.c_double()
        self._check(self._lib.bann_residual_stats(self._h, C.byref(s), C.byref(q)))
        return s.value, q.value

    def residual_shift(self, add: float):
        s, q = C.c_double(), C.c_double()
        self._check(self._lib.bann_residual_shift(self._h, float(add), C.byref(s), C.byref(q)))
        return s.value, q.value

    def residual_to_target(self, b: int):
        self._check(self._lib.bann_residual_to_target(self._h, b))

    def residual_from_target(self, b: int):
        s, q = C.c_double(), C.c_double()
        self._check(self._lib.bann_residual_from_target(self._h, b, C.byref(s), C.byref(q)))
        return s.value, q.value

    def rebuild_targets(self, branches, residual_device_ptr: int = 0):
        """y_b = r + f_b for every listed branch in one launch (r: the context's residual, or a device pointer)."""
        bl = np.ascontiguousarray(branches, dtype=np.int32)
        self._check(self._lib.bann_rebuild_targets(self._h, _ptr(bl, C.c_int32), bl.size,
                                                   C.c_void_p(residual_device_ptr or None)))

    def set_launch_timing(self, enabled: bool):
        self._check(self._lib.bann_set_launch_timing(self._h, 1 if enabled else 0))

    def launch_timing(self, reset: bool = True):
        """(grad_ms, update_ms, grad_launches): averages over the timed leapfrog-session launches."""
        g, u, k = C.c_float(), C.c_float(), C.c_int32()
        self._check(self._lib.bann_launch_timing(self._h, C.byref(g), C.byref(u), C.byref(k), 1 if reset else 0))
        return g.value, u.value, k.value

    def network_timing(self, reset: bool = True):
        """(forward_ms, allreduce_ms, allreduces): averages over the timed network-mode steps."""
        f, a, k = C.c_float(), C.c_float(), C.c_int32()
        self._check(self._lib.bann_network_timing(self._h, C.byref(f), C.byref(a), C.byref(k), 1 if reset else 0))
        return f.value, a.value, k.value

    # ------------------------------------------------------ leapfrog session
    def leapfrog_begin(self, branches: Sequence[int], L: int, max_hamiltonian_error: float = 10.0,
                       step_mode: str = "izmailov", step_factor: float = 1.0, seed: int = 0):
        br = np.ascontiguousarray(branches, dtype=np.int32)
        self._lf_nb = br.size
        self._check(self._lib.bann_leapfrog_begin(self._h, _ptr(br, C.c_int32), br.size, L, max_hamiltonian_error,
                                                  STEP_MODES[step_mode], step_factor, seed))

    def leapfrog_steps(self, k: int):
        self._check(self._lib.bann_leapfrog_steps(self._h, k))

    def leapfrog_end(self):
        st = np.zeros(self._lf_nb, np.int32)
        acc = C.c_int32()
        self._check(self._lib.bann_leapfrog_end(self._h, _ptr(st, C.c_int32), C.byref(acc)))
        return st, acc.value

    def residual_delta_device(self, out_ptr: int):
        """write sum_{accepted b} f_b(theta_L) - f_b(theta_0) (n floats) to a device pointer."""
        self._check(self._lib.bann_leapfrog_residual_delta_device(self._h, C.c_void_p(out_ptr)))

    def residual_delta(self) -> np.ndarray:
        """sum_{accepted b} f_b(theta_L) - f_b(theta_0) as a host array of n floats."""
        out = np.zeros(self.n, np.float32)
        self._check(self._lib.bann_leapfrog_residual_delta(self._h, _ptr(out, C.c_float)))
        return out

    def predictions_device_ptr(self) -> int:
        p = C.POINTER(C.c_float)()
        self._check(self._lib.bann_leapfrog_predictions_device(self._h, C.byref(p)))
        return C.cast(p, C.c_void_p).value or 0

    def profile_session(self, iters: int = 5):
        """(grad_ms, update_ms) average per launch, HIP events on the library stream."""
        g = C.c_float()
        u = C.c_float()
        self._check(self._lib.bann_profile_session(self._h, iters, C.byref(g), C.byref(u)))
        return g.value, u.value

    def synchronize(self):
        self._check(self._lib.bann_synchronize(self._h))
