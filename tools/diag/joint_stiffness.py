"""Stiffness of the network-joint HMC state (bann_network_hmc_step) on a small
synthetic network, CPU only (torch autograd for the Jacobian).

For the joint potential U = lambda_e/2 ||sum_b f_b + bias - y||^2 + sum_b prior_b
the leapfrog with per-parameter Izmailov steps eps_p (ridge_ard.rs:70-117) is
stable while the largest eigenvalue of E H E (E = diag eps, H the Gauss-Newton
Hessian lambda_e J^T J + diag(lambda_p)) stays below 4.  This script prints, for B
branches of the same shape:
  * lam_max(E H E) of one branch alone and of the joint state,
  * the Rayleigh quotient of the joint state along the common mode u = 1/sqrt(n)
    (every branch's output shifted together): lambda_e ||E J^T u||^2,
  * lam_max after the water-filling rule d_p = min(1, t / a_p), a_p = eps_p |g_p|,
    g = J^T 1 (one gradient pass with output error 1), t chosen so that
    lambda_e / n sum_p min(a_p, t)^2 = tau^2,
  * the fraction of parameters whose step the rule leaves unchanged.
    python tools/diag/joint_stiffness.py --branches 50 --n 2000 --m 20
"""
import argparse
import math

import numpy as np
import torch

ap = argparse.ArgumentParser()
ap.add_argument("--branches", type=int, default=50)
ap.add_argument("--n", type=int, default=2000)
ap.add_argument("--m", type=int, default=20)
ap.add_argument("--widths", default="4,4")
ap.add_argument("--factor", type=float, default=1.0)
ap.add_argument("--L", type=int, default=20)
ap.add_argument("--lambda-e", type=float, default=2.0)
ap.add_argument("--tau", type=float, default=1.0)
a = ap.parse_args()
torch.set_default_dtype(torch.float64)
rng = np.random.default_rng(0)
W, S = [int(x) for x in a.widths.split(",")]
n, m, B = a.n, a.m, a.branches


def branch_params():
    w0 = rng.normal(0, math.sqrt(1 / m), (m, W))
    b0 = rng.normal(0, 0.1, W)
    w1 = rng.normal(0, math.sqrt(1 / m), (W, S))
    b1 = rng.normal(0, 0.1, S)
    wo = rng.normal(0, math.sqrt(1 / m), (S, 1))
    return [w0, b0, w1, b1, wo]


def izmailov(params):
    """per-parameter steps from ML ARD precisions (branch_cfg_builder.rs), as bench.py initialises them"""
    w0, b0, w1, b1, wo = params
    lam_w0 = W / np.sum(w0 * w0, axis=1)          # one per input row
    lam_w1 = S / np.sum(w1 * w1, axis=1)
    lam_wo = 1.0 / np.mean(wo * wo)               # the network output precision (order of magnitude)
    lam_b0 = b0.size / np.sum(b0 * b0)
    lam_b1 = b1.size / np.sum(b1 * b1)
    c = a.factor * math.pi / (2 * a.L)
    lam = np.concatenate([np.repeat(lam_w0, W), np.repeat(lam_w1, S), np.full(S, lam_wo), np.full(W, lam_b0),
                          np.full(S, lam_b1)])
    return c / np.sqrt(lam), lam


X = [rng.binomial(2, rng.uniform(0.05, 0.5, m), (n, m)).astype(float) for _ in range(B)]
X = [(x - x.mean(0)) / np.where(x.std(0) > 0, x.std(0), 1) for x in X]
Js, eps, lams = [], [], []
for b in range(B):
    prm = branch_params()
    e, lam = izmailov(prm)
    w0, b0, w1, b1, wo = [torch.tensor(p) for p in prm]
    x = torch.tensor(X[b])

    def f(vec):
        i = 0
        ww0 = vec[i:i + m * W].reshape(W, m).T; i += m * W        # column-major as param_vec
        ww1 = vec[i:i + W * S].reshape(S, W).T; i += W * S
        wwo = vec[i:i + S].reshape(S, 1); i += S
        bb0 = vec[i:i + W]; i += W
        bb1 = vec[i:i + S]; i += S
        a0 = torch.tanh(x @ ww0 + bb0)
        a1 = torch.tanh(a0 @ ww1 + bb1)
        return (a1 @ wwo)[:, 0]

    vec = torch.cat([w0.T.reshape(-1), w1.T.reshape(-1), wo.reshape(-1), b0, b1])
    Js.append(torch.autograd.functional.jacobian(f, vec).numpy())   # n x P_b
    eps.append(e)
    lams.append(lam)
le = a.lambda_e


def lam_max(JE, prior_diag):
    # E H E = le (JE)^T (JE) + diag(eps^2 lam); the prior part is (c pi / 2L)^2 I for Izmailov
    K = le * JE @ JE.T
    return float(np.linalg.eigvalsh(K)[-1]) + float(np.max(prior_diag))


one = [lam_max(J * e[None, :], e * e * lm) for J, e, lm in zip(Js, eps, lams)]
JE = np.concatenate([J * e[None, :] for J, e in zip(Js, eps)], axis=1)
prior = np.concatenate([e * e * lm for e, lm in zip(eps, lams)])
joint = lam_max(JE, prior)
u = np.ones(n) / math.sqrt(n)
cm = le * float(np.sum((JE.T @ u) ** 2))
print(f"B={B} n={n} m={m} W={W} S={S} factor={a.factor} L={a.L}")
print(f"  lam_max(EHE): one branch {np.median(one):.3g} (max {max(one):.3g}), joint {joint:.3g} "
      f"= {joint / np.median(one):.1f} x; common-mode Rayleigh quotient {cm:.3g}")
print(f"  leapfrog stable below 4: one branch omega*eps = {math.sqrt(np.median(one)):.3f}, joint {math.sqrt(joint):.3f}")
# water-filling on the common-mode gains
g = np.concatenate([J.sum(0) for J in Js])        # J^T 1: d(sum_i F_i)/d theta
E = np.concatenate(eps)
A = E * np.abs(g)
Tb = a.tau ** 2 * n / le
if np.sum(A * A) <= Tb:
    t = np.inf
else:
    lo, hi = 0.0, float(A.max())
    for _ in range(100):
        mid = 0.5 * (lo + hi)
        if np.sum(np.minimum(A, mid) ** 2) > Tb:
            hi = mid
        else:
            lo = mid
    t = lo
d = np.minimum(1.0, t / np.maximum(A, 1e-300))
JEd = JE * d[None, :]
joint_d = lam_max(JEd, prior * d * d)
print(f"  water-filling tau={a.tau}: joint lam_max {joint_d:.3g} (omega*eps {math.sqrt(joint_d):.3f}); "
      f"params untouched {np.mean(d >= 1):.3f}, median d {np.median(d):.3f}, mean log2 d {np.mean(np.log2(d)):.2f}")
s_glob = min(1.0, math.sqrt(a.tau ** 2 / joint))
print(f"  uniform scaling to the same joint bound: every step x {s_glob:.4f} (log2 {math.log2(s_glob):.2f})")
