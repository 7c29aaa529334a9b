#!/usr/bin/env python3
"""HMC leapfrog steps/sec on the BASELINE.json cohort (C3: 50k individuals x
500k SNPs x 1k branches of 500 SNPs; D = 1, W = S = 4; RidgeARD, tanh).

One "step" = one full-cohort leapfrog step: a packed gradient evaluation of
every branch (one fused HIP launch) + the fused momentum/position/-H update
(one launch).  The timed region is one whole HMC trajectory of K steps for
every branch: momentum draw + initial gradient, the K steps and the Metropolis
decision; value = K / elapsed.  Each branch runs on its conditional posterior
given the other branches (the target residual + f_b of net.rs:279-280, built
on the device).  Warmup = one untimed trajectory of W steps, then the
roofline's back-to-back launch timing (the GPU clock settles under load).
Genotypes are synthetic (generated on the device), resident in HBM as 2-bit
tile images before the timed region.

  python bench.py [--gpus N --steps K --warmup W]
  (N > 1: one rank per GPU.  Run directly, bench.py starts the N ranks itself
   -- torch.distributed.run as a CHILD process, before anything touches the GPU
   -- and rank 0's JSON line passes through; under an outer
   torch.distributed.run (WORLD_SIZE set) it is one of the ranks.  The 1k
   branches are sharded over the ranks by marker count; a branch-sampler step
   needs no collective (branches share no weights), the timed region ends at a
   barrier and the max over ranks.  --sampler network all-reduces the summed
   branch outputs over RCCL every step.  BANN_DIST_BACKEND=gloo rehearses N
   ranks on one GPU.)

Prints ONE JSON line (rank 0).
"""
import argparse
import ctypes
import glob
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rs-bann_amd"))

CONFIGS = {
    # name: (n, total SNPs, branches, layer_widths)
    "c3": (50_000, 500_000, 1000, [4, 4, 1]),
    "c2": (10_000, 128_000, 64, [4, 4, 1]),
    "small": (8_192, 64_000, 128, [4, 4, 1]),
    # C5 (BASELINE.json configs[4]): 4k branches of 125 SNPs (500k-SNP panel),
    # 100k individuals, W = S = 32: the wide kernel, hidden GEMMs on MFMA
    "c5": (100_000, 500_000, 4000, [32, 32, 1]),
    # C3's cohort with the reference's DEFAULT architecture: hidden and summary
    # widths m_b / 2 (cli.rs:365-375) -- the layered gx path (f32 MFMA GEMMs)
    "c3def": (50_000, 500_000, 1000, [250, 250, 1]),
}
METRIC = "HMC leapfrog steps/sec (whole node), 50k indiv × 500k SNP × 1k branches"
HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md)
F32_MFMA_PEAK_TF = 157.3   # dense f32 MFMA = vector rate (MI355X_MICROARCH.md chip table)
BF16_MFMA_PEAK_TF = 2500.0  # dense bf16 MFMA (spec, no sparsity)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# Izmailov step sizes eps = c pi / (2 sqrt(lambda) L) (ridge_ard.rs:70-117): the
# factor c fixes the trajectory LENGTH L eps, so a c tuned at one L takes steps
# L_ref / L times larger at a shorter L -- past the leapfrog's stability limit on
# the stiff wide / network states (round 3: C5 at c = 0.1 accepted 0.80 at L = 20
# but 0.0005 at L = 10).  The rule: c(L) = c_ref min(1, L / L_ref) -- below the L
# it was tuned at, keep the tuned step size (and shorten the trajectory); above
# it, keep the trajectory length (smaller steps).  (c_ref, L_ref) per line,
# tuned on MI355X (tools/archive/gpu_accept.sh):
TUNED_FACTORS = {
    # (config, sampler, bf16 hidden GEMM): (c_ref, L_ref)
    ("c3", "branch", False): (1.0, 20),       # cli.rs:99-100 default c = 1
    ("c2", "branch", False): (1.0, 20),
    ("small", "branch", False): (1.0, 20),
    ("c3", "sequential", False): (1.0, 20),
    ("c5", "branch", False): (0.1, 20),
    ("c5", "branch", True): (0.02, 20),       # bf16-rounded hidden activations: energy error
    ("c3def", "branch", False): (0.02, 10),
    # the network-joint state with the common-mode step rule (bann_set_network_step_rule,
    # DESIGN.md 7; round 5, 10 trajectories each at L = 20): C3 0.5 accepts 0.9 (1.0: 0.2);
    # C5 0.005 / 0.01 accept 1.0, 0.02 accepts 0.9
    ("c3", "network", False): (0.5, 20),
    ("c5", "network", False): (0.02, 20),
    ("c5", "network", True): (0.01, 20),
}
# ... and without it (--network-step-rule off): the stiffest joint direction -- all branches
# moving the output together -- caps the factor: C3 0.11 accepts, 0.12 diverges; C5 0.0005
# accepts, 0.001 rejects, 0.005 / 0.01 diverge (round 4)
TUNED_FACTORS_NO_RULE = {
    ("c3", "network", False): (0.11, 20),
    ("c5", "network", False): (0.0005, 20),
    ("c5", "network", True): (0.0005, 20),
}


def default_step_factor(config, sampler, bf16, L, rule="common_mode"):
    key = (config, sampler, bf16)
    table = TUNED_FACTORS_NO_RULE if (sampler == "network" and rule == "off") else TUNED_FACTORS
    if key not in table:   # untuned line: the branch sampler's, scaled down for the joint state
        c, l_ref = TUNED_FACTORS.get((config, "branch", bf16), (1.0, 20))
        if sampler == "network":
            c *= 0.1
    else:
        c, l_ref = table[key]
    return c * min(1.0, L / l_ref)


def init_branch_params(rng, m, widths):
    """default init (branch_cfg_builder.rs:180-186): W ~ N(0, 1/m); biases small
    random; ARD ML precisions (308-328); bias ML precisions (264-274)."""
    ins = [m] + widths[:-1]
    ws = [rng.normal(0.0, math.sqrt(1.0 / m), size=(i, o)) for i, o in zip(ins, widths)]
    bs = [rng.normal(0.0, 0.1, size=o) for o in widths[:-1]]
    pv = np.concatenate([w.reshape(-1, order="F") for w in ws] + bs).astype(np.float32)
    prec = []
    for l, w in enumerate(ws[:-1]):
        prec.append(widths[l] / np.sum(w * w, axis=1))
    prec.append(np.array([0.0]))  # output precision: set globally below (architectures.rs:175-185)
    prec += [np.array([b.size / np.sum(b * b)]) for b in bs]
    prec.append(np.array([2.0]))  # error precision (branch_cfg_builder.rs:394)
    return pv, prec, float(np.sum(ws[-1] ** 2))


def cpu_baseline(n, m, widths, sample_branches, sample_steps):
    lib_path = os.path.join(ROOT, "oracle", "libbann_ref_cpu.so")
    if not os.path.exists(lib_path):
        return None
    L = ctypes.CDLL(lib_path)
    f = L.bann_ref_cpu_bench
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    setup, cs = ctypes.c_double(), ctypes.c_double()
    t = f(n, m, widths[0], widths[1], sample_branches, sample_steps, 42, threads, ctypes.byref(setup),
          ctypes.byref(cs))
    if t <= 0:
        return None
    branch_steps_per_s = sample_branches * sample_steps / t
    return dict(branch_steps_per_s=branch_steps_per_s, threads=threads, seconds=t, setup_s=setup.value)


def _fin(x):
    """a float for the JSON line, None where it is not finite (json has no infinity)"""
    return float(x) if math.isfinite(x) else None


def network_check(ctx, dist, dist_dev, world, rank, backend, library_comm, y_net, args, nb, L=20):
    """one network-joint trajectory (bann_network_hmc_step) through the library's
    communicator, timed per phase with HIP events: RCCL's own rank count
    (ncclCommCount), the per-step all-reduce of the summed branch outputs, the
    Metropolis status at half the network sampler's factor for L (the check exercises the
    collective path: at the sampler's own factor one trajectory in ten is rejected, so a
    single decision there says little about the path)."""
    if ctx.comm_info()["kind"] == "none":
        library_comm()
    info = ctx.comm_info()
    factor = 0.5 * default_step_factor(args.config, "network", args.hidden_bf16, L, args.network_step_rule)
    # warm: one untimed trajectory first (it adapts the common-mode rule's factors, the
    # library's auto mode; kernels and the communicator's first collective are loaded),
    # then the timed one, which applies the factors frozen
    ctx.network_hmc_step(y_net, L, bias=0.0, lambda_e=2.0, step_mode="izmailov", step_factor=factor, seed=29)
    ctx.synchronize()
    ctx.set_launch_timing(True)
    if dist is not None:
        dist.barrier()
    t1 = time.perf_counter()
    r = ctx.network_hmc_step(y_net, L, bias=0.0, lambda_e=2.0, step_mode="izmailov", step_factor=factor, seed=31)
    ctx.synchronize()
    el = time.perf_counter() - t1
    ctx.set_launch_timing(False)
    fwd_ms, ar_ms, n_ar = ctx.network_timing(reset=True)
    grad_ms, upd_ms, _ = ctx.launch_timing(reset=True)
    vals = [el, ar_ms, fwd_ms, grad_ms, upd_ms]
    ranks_seen = [float(info["backend_ranks"])]
    if dist is not None:
        import torch
        te = torch.tensor(vals, device=dist_dev, dtype=torch.float64)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        vals = [float(v) for v in te]
        tr = torch.tensor(ranks_seen, device=dist_dev, dtype=torch.float64)
        dist.all_reduce(tr, op=dist.ReduceOp.MIN)
        ranks_seen = [float(tr[0])]
    el, ar_ms, fwd_ms, grad_ms, upd_ms = vals
    rule = ctx.network_step_rule_info()
    rule_state = ctx.network_step_rule_state()
    return {"step_rule": {"kind": args.network_step_rule, "tau": args.network_tau,
                          "timed_trajectory": "frozen" if rule_state["frozen"] else rule_state["mode"],
                          "fraction_scaled": rule["fraction_scaled"], "mode_before": _fin(rule["mode_before"]),
                          "mode_after": _fin(rule["mode_after"])},
            "n_gpus": world, "comm": info["kind"] if info["kind"] == "rccl" else f"callback ({backend})",
            "comm_ranks_reported": int(ranks_seen[0]), "L": L, "step_factor": factor,
            "status": {0: "accepted", 1: "rejected", 2: "rejected_early"}[r["status"]],
            "steps_per_s": L / el, "allreduces": n_ar, "allreduce_us_per_step": 1e3 * ar_ms,
            "allreduce_bytes": 4 * len(y_net), "forward_ms": fwd_ms, "gradient_ms": grad_ms, "update_ms": upd_ms,
            "dH": r["trace"][-1] - r["trace"][0], "branches_per_rank": nb,
            "timing": "HIP events on the library stream, max over ranks; warm (after one untimed trajectory)"}


def launch_ranks(nproc: int) -> int:
    """`bench.py --gpus N` run directly (no WORLD_SIZE): start the N ranks as
    `torch.distributed.run` in a child process -- never exec, and nothing here
    touches the GPU -- wait for it and return its exit code.  The ranks inherit
    stdout, so rank 0's JSON line is this command's output."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only (RCCL across processes)
    env.setdefault("OMP_NUM_THREADS", "1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    log(f"bench.py: launching {nproc} ranks: {' '.join(cmd[1:])}")
    return subprocess.call(cmd, env=env)


def check_launch(dist, world, rank, n=4096, nbranches=1000):
    """--check-launch: the multi-rank plumbing without a GPU (CPU test): every
    rank takes its marker-balanced branch shard (bann_shard_branches) and runs
    the library's residual exchange step (bann_residual_update_host: the sum
    over ranks of the local residual changes through the communicator's
    all-reduce, then residual -= sum -- what bann_exchange_residual does for a
    callback communicator) on a rank-specific change; rank 0 prints one JSON line."""
    import torch
    from bann.distributed import TorchAllreduce, residual_update, shard_ranges
    lo, hi = shard_ranges([500] * nbranches, world)[rank]
    base = np.linspace(-1.0, 1.0, n, dtype=np.float32)
    delta = (np.arange(n, dtype=np.float32) % 7) * np.float32(rank + 1)   # this rank's local change
    res = residual_update(base.copy(), delta, TorchAllreduce(dist) if dist is not None else None)
    want = base - (np.arange(n, dtype=np.float32) % 7) * np.float32(world * (world + 1) / 2)
    rec = torch.tensor([rank, lo, hi, float(np.max(np.abs(res - want)))], dtype=torch.float64)
    if dist is not None:
        recs = [torch.zeros_like(rec) for _ in range(world)]
        dist.all_gather(recs, rec)
    else:
        recs = [rec]
    if rank == 0:
        print(json.dumps({"check_launch": True, "n_gpus": world,
                          "ranks": [int(r[0]) for r in recs],
                          "shards": [[int(r[1]), int(r[2])] for r in recs],
                          "exchange_max_err": max(float(r[3]) for r in recs),
                          "parallelism": f"branch-shard x{world}"}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)   # L = 100: the reference default integration length (mcmc_cfg.rs:38)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--step-factor", type=float, default=None,
                    help="Izmailov factor c; default 1.0 (cli.rs:99-100), 0.1 for c5, 0.02 for c3def (wide branches: acceptance > 0.6 at L = 100)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-branches", type=int, default=None)   # default 96 (c3def: 4), capped at the branch count
    ap.add_argument("--cpu-sample-steps", type=int, default=None)      # default 16 (c3def: 2)
    ap.add_argument("--profile-iters", type=int, default=20)
    ap.add_argument("--no-launch-timing", action="store_true",
                    help="no HIP events around the timed trajectory's launches (roofline from the back-to-back session)")
    ap.add_argument("--emulate-shard", type=int, default=0,
                    help="profiling only: run rank 0's shard of an N-GPU job on this one GPU, no collective")
    ap.add_argument("--hidden-bf16", action="store_true",
                    help="wide kernel: hidden GEMMs on bf16 MFMA (C5's bf16 vs fp32 comparison)")
    ap.add_argument("--sampler", default="branch", choices=["branch", "network", "sequential"],
                    help="branch: every branch's trajectory against the sweep-start residual, one residual "
                         "exchange per trajectory (default); network: one HMC state over all branches, the summed "
                         "branch outputs all-reduced every leapfrog step (bann_network_hmc_step); sequential: the "
                         "reference's own sweep order, one branch at a time against the refreshed residual "
                         "(bann_net_train, Net::train net.rs:201-358), one GPU")
    ap.add_argument("--no-network-check", action="store_true",
                    help="skip the untimed network-joint trajectory through the library's RCCL communicator "
                         "(a 1-rank one at N = 1) that runs before the warmup and is reported in the line "
                         "(network_check)")
    ap.add_argument("--network-step-rule", default="common_mode", choices=["common_mode", "adaptive", "off"],
                    help="network-joint step sizes: the common-mode water-filling rule (bann_set_network_step_rule; "
                         "default: adapted during the warmup, frozen for the timed and acceptance trajectories), "
                         "adaptive (re-adapted before every trajectory) or the per-branch Izmailov steps as they are")
    ap.add_argument("--network-tau", type=float, default=1.0,
                    help="common-mode rule: omega eps of the network's common mode after the rule")
    ap.add_argument("--accept-trajectories", type=int, default=None,
                    help="untimed trajectories after the timed one whose acceptance is reported beside it "
                         "(default 4 for --sampler network: one Metropolis decision per trajectory)")
    ap.add_argument("--check-launch", action="store_true",
                    help="no GPU: run the N-rank launch, shard and the library's residual exchange step only (CPU test)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    backend = os.environ.get("BANN_DIST_BACKEND", "gloo" if args.check_launch else "nccl")   # gloo: N ranks on one GPU
    dist_dev = "cuda" if backend == "nccl" else "cpu"
    if world > 1:
        import torch
        import torch.distributed as dist_mod
        if not args.check_launch:
            local_rank = local_rank % max(torch.cuda.device_count(), 1)
            torch.cuda.set_device(local_rank)
        dist_mod.init_process_group(backend, init_method="env://")
        dist = dist_mod
    if args.check_launch:
        check_launch(dist, world, rank)
        if dist is not None:
            dist.destroy_process_group()
        return

    from bann import BannContext
    from bann.distributed import TorchAllreduce, comm_unique_id, shard_ranges

    n, M_total, B_total, widths = CONFIGS[args.config]
    if args.step_factor is None:
        args.step_factor = default_step_factor(args.config, args.sampler, args.hidden_bf16, args.steps,
                                               args.network_step_rule)
    heavy = widths[0] > 32   # gx-path configs: minutes of CPU per branch-step at full size
    if args.cpu_sample_branches is None:
        args.cpu_sample_branches = 4 if heavy else 96
    if args.cpu_sample_steps is None:
        args.cpu_sample_steps = 2 if heavy else 24  # ~10-15 s of CPU work at C3
    m_b = M_total // B_total
    b0, b1 = shard_ranges([m_b] * B_total, max(world, args.emulate_shard))[rank]   # contiguous, balanced by markers
    nb = b1 - b0

    t_setup = time.time()
    ctx = BannContext(local_rank)
    # this rank's markers only (uniform contiguous grouping, uniform.rs:11-23)
    ctx.synthetic_genotypes(n, nb * m_b, seed=1000003 * (rank + 1))
    for k in range(nb):
        ctx.add_branch(np.arange(k * m_b, (k + 1) * m_b, dtype=np.int32), widths, "tanh", "ridge_ard")
    ctx.finalize(free_raw=True)
    # the library default (auto): the first trajectory adapts the common-mode factors, every later
    # one applies them frozen (state-independent step sizes); "adaptive" re-adapts before every one
    ctx.set_network_step_rule({"common_mode": "auto", "adaptive": "adaptive", "off": "off"}[args.network_step_rule],
                              args.network_tau)
    path = ctx.kernel_path(0)
    assert path == ("layered" if heavy else "wide" if widths[0] > 4 else "fused" if m_b <= 512 else "fused_large")
    assert all(ctx.kernel_path(k) == path for k in range(nb))
    wide = path in ("wide", "layered")   # MFMA-bound: hidden-layer GEMMs
    if args.hidden_bf16:
        ctx.set_hidden_gemm_bf16(True)
    params, precs, out_ss = [], [], 0.0
    for k in range(nb):
        rng = np.random.default_rng(b0 + k)
        pv, prec, ss = init_branch_params(rng, m_b, widths)
        params.append(pv)
        precs.append(prec)
        out_ss += ss
    tot = np.array([out_ss, float(nb)])
    if dist is not None:
        import torch
        tt = torch.tensor(tot, device=dist_dev)
        dist.all_reduce(tt)
        tot = tt.cpu().numpy()
    out_prec = tot[1] / tot[0]
    fsum = np.zeros(n, np.float64)
    for k in range(nb):
        ctx.set_params(k, params[k])
    preds = ctx.predict_many(list(range(nb)))   # one packed launch
    fsum += preds.sum(axis=0, dtype=np.float64)
    if dist is not None:
        import torch
        tt = torch.tensor(fsum, device=dist_dev)
        dist.all_reduce(tt)
        fsum = tt.cpu().numpy()
    # phenotype y = sum_b f_b + noise at h^2 = 0.5; residual = noise; each branch
    # is fitted to its partial residual residual + f_b (net.rs:279-280)
    # residual noise at the error precision's default 2.0 (branch_cfg_builder.rs:394):
    # Var(noise) = 1 / 2, the value the error precision's Gibbs draw
    # (sample_error_precision, net.rs:272) is consistent with, whatever the summed
    # output's scale (a W = 250 cohort's sum is ~40x a W = 4 one's)
    noise = np.random.default_rng(7).normal(0.0, math.sqrt(0.5), size=n)
    for k in range(nb):
        prec = precs[k]
        prec[len(widths) - 1] = np.array([out_prec])
        ctx.set_precisions(k, np.concatenate(prec).astype(np.float32))
    # the sweep's residual y - sum_b f_b (net.rs:279-300) lives on the device; every
    # branch target y_b = residual + f_b is built there in one launch
    ctx.residual_set(noise.astype(np.float32))
    ctx.rebuild_targets(list(range(nb)))
    del preds
    ctx.synchronize()
    setup_s = time.time() - t_setup

    # every rank's branch count must be its shard_ranges entry, every rank present once
    # (a mis-ranked launch -- duplicate RANKs, a wrong WORLD_SIZE -- exits non-zero)
    if dist is not None:
        import torch
        sh = torch.zeros(2 * world, device=dist_dev, dtype=torch.float64)
        sh[rank], sh[world + rank] = float(nb), 1.0
        dist.all_reduce(sh)
        want = [float(e - s_) for s_, e in shard_ranges([m_b] * B_total, max(world, args.emulate_shard))[:world]]
        got, seen_r = [float(v) for v in sh[:world]], [float(v) for v in sh[world:]]
        if seen_r != [1.0] * world or got != want:
            log(f"rank {rank}: shard check failed: branches per rank {got}, shard_ranges {want}, ranks seen {seen_r}")
            sys.stdout.flush()
            os._exit(5)

    def library_comm():
        """the library's communicator: RCCL over xGMI (one GPU per rank), or a gloo
        all-reduce callback when rehearsing N ranks on one GPU"""
        if dist is None:   # one rank: a 1-rank RCCL communicator
            ctx.comm_init_rccl(comm_unique_id(), 1, 0)
        elif backend == "nccl":
            import torch
            idt = torch.zeros(128, dtype=torch.uint8, device=f"cuda:{local_rank}")
            if rank == 0:
                idt.copy_(torch.frombuffer(bytearray(comm_unique_id()), dtype=torch.uint8))
            dist.broadcast(idt, 0)
            ctx.comm_init_rccl(bytes(idt.cpu().numpy()), world, rank)
        else:
            ctx.comm_callback(TorchAllreduce(dist), world, rank)
        ctx.synchronize()

    if dist is not None and args.sampler == "network":   # the per-step all-reduce needs it in the timed region
        library_comm()
    branches = list(range(nb))
    y_net = (noise + fsum).astype(np.float32)

    net, seen = None, [0.0]
    if args.sampler == "sequential":
        if world > 1:
            raise SystemExit("--sampler sequential is the single-device driver (Net::train)")
        from bann.net import MCMCConfig, Net
        net = Net(ctx, seed=5)
        net.set_global(2.0, float(out_prec))

    def trajectory(L, seed):
        """one HMC trajectory of L leapfrog steps.  branch sampler: every branch of
        this rank (momentum draw + initial gradient, L fused steps, Metropolis) on
        its conditional posterior given the other branches at the sweep start (the
        target y_b = residual + f_b of net.rs:279-280, built on the device).  The
        targets are NOT rebuilt between trajectories: a simultaneous (Jacobi)
        update of 1000 overlapping branches (2M parameters, n = 50k) overshoots the
        residual -- measured: ||r||^2 +70 % after one trajectory and every later
        trajectory rejected early (tools/archive/diag_c3.py) -- so the
        residual bookkeeping of a sweep belongs to the sequential driver
        (--sampler sequential, the reference's Gauss-Seidel order) and the
        network sampler.  network sampler: one HMC state over all branches of all
        ranks, the summed outputs all-reduced every step (bann_network_hmc_step)."""
        if args.sampler == "sequential":   # one sweep: every branch one L-step trajectory, in shuffled order
            net.train(y_net, MCMCConfig(hmc_step_size_factor=args.step_factor, hmc_integration_length=L,
                                        chain_length=1, burn_in=1))
            before, seen[0] = seen[0], float(net.summary()["num_accepted"])
            return seen[0] - before
        if args.sampler == "network":
            # the Metropolis uniform: drawn by the library on rank 0 (seed) and shared
            r = ctx.network_hmc_step(y_net, L, bias=0.0, lambda_e=2.0, step_mode="izmailov",
                                     step_factor=args.step_factor, seed=seed)
            if os.environ.get("BANN_BENCH_TRACE"):   # diagnostics: the network -H trace on stderr
                log(json.dumps({"seed": seed, "status": int(r["status"]), "trace": [float(v) for v in r["trace"]]}))
            return float(r["status"] == 0) * nb
        ctx.leapfrog_begin(branches, L, 10.0, "izmailov", args.step_factor, seed=seed)
        ctx.leapfrog_steps(L)
        status, acc = ctx.leapfrog_end()
        return acc

    # C4's collective, checked before anything is timed and reported INSIDE the
    # line: one network-joint trajectory through the library's communicator (RCCL
    # over xGMI at N > 1: the per-step all-reduce of the summed branch outputs),
    # from the generating state (y = sum_b f_b + noise), at the network sampler's
    # factor for its L.  A stalled collective ends the run with a non-zero exit
    # (watchdog), an error likewise; the line is never printed without it.
    netcheck = None
    if args.sampler == "branch" and not args.no_network_check:
        import threading
        wd = threading.Timer(180.0, lambda: (log(f"network_check: rank {rank}: collective stalled"), os._exit(3)))
        wd.daemon = True
        wd.start()
        try:
            netcheck = network_check(ctx, dist, dist_dev, world, rank, backend, library_comm, y_net, args, nb)
        except Exception as exc:  # noqa: BLE001
            log(f"network_check: rank {rank}: {exc!r}")
            sys.stdout.flush()
            os._exit(4)
        wd.cancel()
        if rank == 0:
            log(json.dumps({"network_check": netcheck}))
        # a mis-ranked run must not publish a line: RCCL's own rank count (MIN over ranks)
        # has to be the launch's world size
        if netcheck["comm_ranks_reported"] != world:
            log(f"network_check: the communicator reports {netcheck['comm_ranks_reported']} ranks, "
                f"the launch has {world}")
            sys.stdout.flush()
            os._exit(5)
        # the library leaves every branch's target at its Gibbs target of the state the
        # check ended in (accepted: its last step; otherwise theta_0) and the device
        # residual at y - sum_b f_b (include/bann.h): the branch line samples from there

    # warmup: a full trajectory of W steps (loads every kernel), then the
    # roofline's back-to-back launch timing (bann_profile_session: a 2-step
    # trajectory whose gradient and update launches are repeated profile_iters
    # times without changing the chain) -- untimed work that also lets the GPU's
    # clock settle under the HBM load before the timed trajectory (the first
    # ~10 gradient launches after a light phase run up to 30 % slow while the
    # power controller settles: profiles/r03a_transient.md).
    # The session is a branch-sampler trajectory (every branch against its own
    # target: a Jacobi step of the whole network), which the network and
    # sequential samplers must not see: the network sampler times its own
    # gradient launches instead and runs no session; the sequential driver runs it
    # first and puts the parameters back (the warmup sweep then re-settles the clock).
    def b2b_session(restore):
        snap = [ctx.get_params(b) for b in branches] if restore else None
        ctx.leapfrog_begin(branches, 2, 10.0, "izmailov", args.step_factor, seed=99 + rank)
        r = ctx.profile_session(args.profile_iters)
        ctx.leapfrog_end()
        if restore:
            for b in branches:
                ctx.set_params(b, snap[b])
        return r
    b2b_grad_ms = b2b_upd_ms = None
    if args.sampler == "sequential" or (args.sampler == "network" and args.no_launch_timing):
        b2b_grad_ms, b2b_upd_ms = b2b_session(restore=True)
    if args.warmup:
        trajectory(args.warmup, seed=7 + rank)
    if args.sampler == "network":
        # the network line has no back-to-back session (it would move the joint state): one more
        # untimed trajectory of K steps (burn-in) settles the GPU clock under the trajectory's own
        # load -- without it the timed trajectory's first gradient launches ran 1.3-1.6 ms against
        # 1.10 later (profiles/r06c_net_summary.md, the power controller's transient)
        trajectory(args.steps, seed=5 + rank)
    # network sampler, common-mode rule (auto): the warmup trajectory adapted the step factors
    # (burn-in); the timed and the acceptance trajectories apply them frozen -- step sizes
    # independent of each trajectory's start, as HMC's reversibility asks
    if args.sampler == "branch":
        b2b_grad_ms, b2b_upd_ms = b2b_session(restore=False)
    timing = args.sampler in ("branch", "network") and not args.no_launch_timing
    if timing:   # HIP events around every gradient / update launch of the timed trajectory
        ctx.launch_timing(reset=True)
        ctx.set_launch_timing(True)
    ctx.synchronize()
    if dist is not None:
        torch.cuda.synchronize()
        dist.barrier()
    t0 = time.perf_counter()
    acc = trajectory(args.steps, seed=11 + rank)   # timed: one whole trajectory of K steps
    ctx.synchronize()
    if dist is not None:
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if timing:
        ctx.set_launch_timing(False)
        grad_ms, upd_ms, n_launch = ctx.launch_timing(reset=True)
        if args.sampler == "network":   # the timed trajectory's forward-only launches and all-reduces
            net_fwd_ms, net_ar_ms, net_n_ar = ctx.network_timing(reset=True)
    else:
        grad_ms, upd_ms, n_launch = b2b_grad_ms, b2b_upd_ms, 0
    if dist is not None:
        te = torch.tensor([elapsed], device=dist_dev, dtype=torch.float64)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        elapsed = float(te.item())
        ta = torch.tensor([acc, nb], device=dist_dev, dtype=torch.float64)
        dist.all_reduce(ta)
        acc_all, nb_all = float(ta[0]), float(ta[1])
    else:
        acc_all, nb_all = float(acc), float(nb)
    # acceptance over more (untimed) trajectories: the network sampler takes ONE
    # Metropolis decision per trajectory, so a single trajectory says 0 or 1
    n_extra = args.accept_trajectories if args.accept_trajectories is not None else (
        4 if args.sampler == "network" else 0)
    accs = [acc / nb]
    for i in range(n_extra):
        accs.append(trajectory(args.steps, seed=101 + 7 * i + rank) / nb)
    if dist is not None and n_extra:
        ta = torch.tensor(accs, device=dist_dev, dtype=torch.float64)
        dist.all_reduce(ta)
        accs = [float(v) / world for v in ta]

    workload = (f"{args.config}: {B_total} branches x {m_b} SNPs, n={n}, D=1 W={widths[0]} S={widths[1]}, RidgeARD, "
                "tanh, Izmailov step sizes" + (", bf16 hidden GEMM" if args.hidden_bf16 else "") +
                (", network-joint sampler (per-step all-reduce)" if args.sampler == "network" else "") +
                (", sequential Net::train sweep (one branch at a time)" if args.sampler == "sequential" else ""))
    wx_planes = path == "wide" and not args.hidden_bf16 and os.environ.get("BANN_WX_EXACT", "0") in ("", "0")
    # fxl shapes of 17..32 chunks run the head-wave kernel (kernels_fx.hip fxh_takes)
    nch_b = -(-m_b // 64)
    fxh = nch_b <= 32 and -(-nch_b // 4) >= 5 and os.environ.get("BANN_FXL_HEAD", "1") != "0"
    kernel_name = {"wide": "k_fused_grad_wx3" if wx_planes else "k_fused_grad_wx", "fused": "k_fused_grad_fx",
                   "fused_large": "k_fused_grad_fxh" if fxh else "k_fused_grad_fxl", "layered": "k_gx_gemm"}[path]
    # ---- kernel timing for the roofline: HIP events on the library stream around
    # the timed trajectory's own gradient launches (bann_set_launch_timing); the
    # back-to-back figure of the warmup session is reported beside it ----
    # algorithmic bytes per gradient launch: the genotype block of every branch
    # read once at its information content -- 2 bits per genotype, i.e. the
    # .bed payload size ceil(n/4) * m_b (bed.rs:193-245) -- plus the per-branch
    # f32 targets (4 n B).  O(P) parameter / partial traffic is < 0.5 % and not
    # counted.  (The int8 layout of the generic path would be 4x this; the
    # fused kernel streams the 2-bit codes, so counting int8 bytes would
    # overstate the achieved bandwidth 4x.)
    x_bytes = ((n + 3) // 4) * m_b * nb
    # network sampler on the fx path: every branch reads the one network error vector
    # (DevState::nete), L2-resident, instead of a target row of its own
    net_err = args.sampler == "network" and path == "fused" and os.environ.get("BANN_NET_ERR", "1") != "0"
    y_bytes = 4 * n * (1 if net_err else nb)
    alg_bytes = x_bytes + y_bytes
    achieved = alg_bytes / (grad_ms * 1e-3) / 1e9
    # wide branches: the dominant work is the hidden-layer GEMMs on MFMA --
    # forward Z1 = A0 W1, error propagation err0 = delta1 W1^T and dW1 = A0^T delta1,
    # 2 n W S flops each per branch (branch_sampler.rs:760-771, 844-866)
    hidden_flops = 3 * 2 * n * widths[0] * widths[1] * nb
    if path == "layered":   # gx: every GEMM on the f32 MFMA -- masked layer forward + dW0, hidden GEMMs
        hidden_flops += 2 * 2 * n * m_b * widths[0] * nb
    # the masked layer on the i8 MFMA: W0 and delta0 as 4 digits, forward + backward
    i8_ops = 2 * 2 * n * m_b * 4 * widths[0] * nb
    # HBM traffic per gradient launch, from the committed PMC pass of the same
    # workload (tools/profile_round.sh; a --pmc run cannot time itself)
    traffic, traffic_src, mfma_pmc = None, None, None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")), reverse=True):
        pm = json.load(open(f))
        if world == 1 and not args.emulate_shard and pm.get("config", "").split(":")[0] == workload.split(":")[0] and pm.get("kernel", "").startswith(f"void {kernel_name}<"):
            traffic, traffic_src = pm["traffic_bytes_per_launch"], os.path.relpath(f, ROOT)
            mfma_pmc = pm.get("mfma")
            break

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sample_b = min(args.cpu_sample_branches, B_total)
        c = cpu_baseline(n, m_b, widths, sample_b, args.cpu_sample_steps)
        if c is not None:
            cpu = {"value": c["branch_steps_per_s"] / B_total, "unit": "leapfrog steps/s",
                   "cores": c["threads"], "kind": "port",
                   "sample": f"{sample_b} branches x {args.cpu_sample_steps} leapfrog steps at "
                             f"n={n}, m_b={m_b}, widths={widths} (C restatement of the reference op order, f32, "
                             f"X read 3x per step), extrapolated x{B_total}/{sample_b} branches; "
                             f"{c['seconds']:.1f}s of CPU work"}

    steps_per_s = args.steps / elapsed
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": steps_per_s,
            "unit": "leapfrog steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "2-bit genotype codes x f32 params (i8 MFMA digits, exact int32 accumulate, f32 head)",
            "data": "synthetic (device-generated Binomial(2,p) genotypes, random-init branches)",
            "config": {"workload": workload,
                       "n": n, "snps": M_total, "branches": B_total, "layer_widths": widths,
                       "branches_per_gpu": nb, "parallelism": f"branch-shard x{world}"},
            "roofline": ({"bound": "mfma", "achieved": hidden_flops / (grad_ms * 1e-3) / 1e12,
                          "peak": BF16_MFMA_PEAK_TF if args.hidden_bf16 else F32_MFMA_PEAK_TF, "unit": "TFLOP/s",
                          "frac": hidden_flops / (grad_ms * 1e-3) / 1e12 /
                          (BF16_MFMA_PEAK_TF if args.hidden_bf16 else F32_MFMA_PEAK_TF),
                          "basis": ("f32-equivalent GEMM flops 4 n m W + 6 n W S per branch per launch (the whole "
                                    "gradient evaluation: FWD0, FWD1, BWD1, GRAD1, GRAD0) against the f32 MFMA peak "
                                    "(the parity-exact BANN_GX_EXACT=1 path's ceiling); executed on the bf16 MFMA: "
                                    "the masked layer with the f32 operand as three bf16 planes (3 products), the "
                                    "hidden layers with both operands as three planes (6 products), see "
                                    "bf16_pipe_frac") if path == "layered" else
                                   ("f32-equivalent hidden-layer GEMM flops 6 n W S per branch per launch against "
                                    "the f32 MFMA peak (the BANN_WX_EXACT=1 path's ceiling); executed on the bf16 "
                                    "MFMA with both operands as three bf16 planes (6 products, f32-accurate), see "
                                    "bf16_pipe_frac") if wx_planes else
                                   "hidden-layer GEMM flops 6 n W S per branch per launch",
                          **({"bf16_pipe_frac": (3 * 2 * 2 * n * m_b * widths[0] + 6 * 3 * 2 * n * widths[0] * widths[1])
                              * nb / (grad_ms * 1e-3) / 1e12 / BF16_MFMA_PEAK_TF} if path == "layered" else
                             {"bf16_pipe_frac": 6 * hidden_flops / (grad_ms * 1e-3) / 1e12 / BF16_MFMA_PEAK_TF}
                             if wx_planes else {}),
                          "i8_mfma_tops": i8_ops / (grad_ms * 1e-3) / 1e12,
                          "mfma_busy_pmc": (mfma_pmc or {}).get("mfma_busy_per_simd_cycle"),
                          "hbm_GBps": achieved} if wide else
                         {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": achieved / HBM_PEAK_GBS}) | {"traffic": traffic,
                         "traffic_unit": "bytes per launch", "traffic_source": traffic_src,
                         "kernel": kernel_name, "kernel_ms": grad_ms,
                         "kernel_ms_source": (f"HIP events around the {n_launch} gradient launches of the timed "
                                              "trajectory" if n_launch else "back-to-back launches (bann_profile_session)"),
                         "kernel_ms_back_to_back": b2b_grad_ms, "alg_bytes_per_launch": alg_bytes,
                         "packed_bytes_per_launch": ctx.packed_genotype_bytes,
                         "alg_bytes_basis": ("2-bit genotypes (n*m_b/4) per branch + the 4n-byte network error once"
                                             if net_err else "2-bit genotypes (n*m_b/4) + 4n target bytes per branch"),
                         "update_kernel_ms": upd_ms},
            "cpu_baseline": cpu,
            "accept_rate": acc_all / nb_all,
            **({"accept_rate_trajectories": {"trajectories": len(accs), "rate": float(np.mean(accs))}}
               if n_extra else {}),
            "step_factor": args.step_factor,
            "sampler": args.sampler,
            "setup_s": setup_s,
        }
        if args.sampler == "network":
            if timing:
                out["network_timing"] = {"forward_ms": net_fwd_ms, "allreduce_us_per_step": 1e3 * net_ar_ms,
                                         "allreduces": net_n_ar,
                                         "source": "HIP events around the timed trajectory's launches"}
            rule = ctx.network_step_rule_info()
            out["network_step_rule"] = {"kind": args.network_step_rule, "tau": args.network_tau,
                                        "fraction_scaled": rule["fraction_scaled"],
                                        "mode_before": _fin(rule["mode_before"]),
                                        "mode_after": _fin(rule["mode_after"])}
        if netcheck is not None:
            out["network_check"] = netcheck
        if args.emulate_shard:
            out["emulated_shard_of"] = args.emulate_shard   # not a whole-job number: one rank's shard
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
