"""Network-joint HMC (bann_network_hmc_step): one HMC state over every branch,
the per-step sum of branch outputs exchanged over the ranks.

  * one rank: trajectory, -H trace, status and final parameters match the
    oracle restatement (bann_oracle.network_hmc_step);
  * two ranks on one GPU (two processes, two contexts, a gloo all-reduce
    callback as the communicator -- RCCL needs one GPU per rank): the sharded
    run reproduces the one-rank run (same status, -H trace within 1e-5, same
    final parameters)."""
import os
import socket

import numpy as np
import pytest

import bann_oracle as O
from helpers import f32_branch, norm_rel, x_std

pytestmark = pytest.mark.gpu

SHAPES = [(60, [4, 4, 1], "ridge_ard"), (40, [8, 8, 1], "lasso_base"), (700, [4, 4, 1], "ridge_base"),
          (30, [6, 5, 3, 1], "lasso_ard")]


def _problem(seed=5, n=800):
    rng = np.random.default_rng(seed)
    M = sum(m for m, _, _ in SHAPES)
    g = O.synthetic_genotypes(rng, n, M)
    specs, off = [], 0
    for m, w, prior in SHAPES:
        specs.append(dict(snps=np.arange(off, off + m, dtype=np.int32),
                          branch=f32_branch(O.random_branch(rng, m, w, prior=prior))))
        off += m
    return rng, g, specs


def _context(g, specs, branches):
    from bann import BannContext
    ctx = BannContext(0)
    ctx.upload_genotypes(g)
    for b in branches:
        br = specs[b]["branch"]
        ctx.add_branch(specs[b]["snps"], br.layer_widths, br.act, br.prior)
    ctx.finalize()
    for i, b in enumerate(branches):
        br = specs[b]["branch"]
        ctx.set_params(i, O.param_vec(br.weights, br.biases))
        ctx.set_precisions(i, O.precision_vec(br))
    return ctx


def _draws(rng, specs, L):
    eps, mom = [], []
    for s in specs:
        ew, eb = O.izmailov_step_sizes(s["branch"], 0.3, L)
        eps.append(O.param_vec(ew, eb).astype(np.float32))
        mom.append(rng.normal(size=s["branch"].num_params).astype(np.float32))
    return eps, mom


def _check_final_targets(ctx, brs, Xs, y, bias):
    """the state bann_network_hmc_step leaves (include/bann.h): the device residual is
    y - bias - sum_b f_b of the final parameters (accepted or restored) and every
    branch's target is its Gibbs target f_b - e, so rss against it is the network's"""
    r = y - bias - sum(O.predict(br, X) for br, X in zip(brs, Xs))
    assert norm_rel(ctx.residual_get(), r) < 1e-5
    rss = float(np.sum(r * r))
    for b in range(len(brs)):
        assert abs(ctx.rss(b) - rss) <= 1e-5 * rss, (b, ctx.rss(b), rss)


def test_network_hmc_matches_oracle():
    rng, g, specs = _problem()
    n, L = g.shape[1], 6
    ctx = _context(g, specs, range(len(specs)))
    mu, sd = ctx.genotype_stats()
    Xs = [x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]]) for s in specs]
    f = sum(O.predict(s["branch"], X) for s, X in zip(specs, Xs))
    y = (f + rng.normal(scale=0.7, size=n)).astype(np.float32).astype(np.float64)
    bias, le = 0.25, 1.5
    for u in (0.4, 0.999999):
        eps, mom = _draws(rng, specs, L)
        res = ctx.network_hmc_step(y, L, bias=bias, lambda_e=le, eps=np.concatenate(eps),
                                   momentum=np.concatenate(mom), u=u)
        brs = [s["branch"].copy() for s in specs]
        out = O.network_hmc_step(brs, Xs, y, bias, le, [e.astype(np.float64) for e in eps],
                                 [p.astype(np.float64) for p in mom], L, 10.0, u)
        assert res["status"] == out["status"], (res["status"], out["status"])
        tr = np.asarray(out["trace"])
        assert np.all(np.abs(res["trace"][: tr.size] - tr) <= 1e-5 * np.maximum(1.0, np.abs(tr))), (res["trace"], tr)
        for b, br in enumerate(brs):
            assert norm_rel(ctx.get_params(b), O.param_vec(br.weights, br.biases)) < 1e-5, b
        _check_final_targets(ctx, brs, Xs, y, bias)
        for s, br in zip(specs, brs):
            s["branch"] = f32_branch(br)
            s["branch"].error_precision = specs[0]["branch"].error_precision
    ctx.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_worker(rank, world, port, out, u=0.5):
    import torch.distributed as dist
    from bann.distributed import TorchAllreduce, shard_ranges
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng, g, specs = _problem(seed=9)
    n, L = g.shape[1], 5
    y = rng.normal(size=n).astype(np.float32)
    eps, mom = _draws(rng, specs, L)
    lo, hi = shard_ranges([m for m, _, _ in SHAPES], world)[rank]
    ctx = _context(g, specs, range(lo, hi))
    if world > 1:
        ctx.comm_callback(TorchAllreduce(dist), world, rank)
    res = ctx.network_hmc_step(y, L, bias=-0.1, lambda_e=0.8, eps=np.concatenate(eps[lo:hi]),
                               momentum=np.concatenate(mom[lo:hi]), u=u, seed=17)
    out[rank] = dict(status=res["status"], trace=res["trace"],
                     params=[ctx.get_params(i) for i in range(hi - lo)], lo=lo)
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("u", [0.5, None])
def test_network_hmc_two_ranks_match_one(u):
    """u = None: the library draws the Metropolis uniform on rank 0 and shares it
    through the -H all-reduce, so both ranks take the one-rank decision."""
    import torch.multiprocessing as mp
    results = {}
    for world in (1, 2):
        mgr = mp.Manager()
        out = mgr.dict()
        mp.spawn(_rank_worker, args=(world, _free_port(), out, u), nprocs=world, join=True)
        results[world] = dict(out)
    one, two = results[1][0], results[2]
    assert two[0]["status"] == two[1]["status"] == one["status"]
    assert np.array_equal(two[0]["trace"], two[1]["trace"])   # identical network decision on every rank
    assert np.all(np.abs(two[0]["trace"] - one["trace"]) <= 1e-5 * np.maximum(1.0, np.abs(one["trace"])))
    params = two[0]["params"] + two[1]["params"]
    for b, pv in enumerate(params):
        assert norm_rel(pv, one["params"][b]) < 1e-5, b


def test_rccl_one_rank_communicator():
    """the library's RCCL communicator (bann_comm_unique_id + bann_ctx_comm_init)
    at world size 1, on the GPU: RCCL reports one rank, and every collective path
    -- the network trajectory's per-step f32 all-reduce of the summed branch
    outputs, its f64 -H / uniform all-reduce, and the device residual exchange
    of a leapfrog session -- gives the bits of the same calls with no
    communicator, and the oracle's trajectory."""
    from bann.distributed import comm_unique_id
    rng, g, specs = _problem(seed=13)
    n, L = g.shape[1], 5
    plain = _context(g, specs, range(len(specs)))
    rccl = _context(g, specs, range(len(specs)))
    assert plain.comm_info()["kind"] == "none"
    rccl.comm_init_rccl(comm_unique_id(), 1, 0)
    info = rccl.comm_info()
    assert info == dict(kind="rccl", nranks=1, rank=0, backend_ranks=1), info
    mu, sd = plain.genotype_stats()
    Xs = [x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]]) for s in specs]
    y = rng.normal(size=n).astype(np.float32)
    eps, mom = _draws(rng, specs, L)
    # injected draws: both contexts and the oracle
    brs = [s["branch"].copy() for s in specs]
    rccl.set_launch_timing(True)
    r0 = plain.network_hmc_step(y, L, bias=0.1, lambda_e=0.9, eps=np.concatenate(eps), momentum=np.concatenate(mom),
                                u=0.3)
    r1 = rccl.network_hmc_step(y, L, bias=0.1, lambda_e=0.9, eps=np.concatenate(eps), momentum=np.concatenate(mom),
                               u=0.3)
    rccl.set_launch_timing(False)
    fwd_ms, ar_ms, n_ar = rccl.network_timing()
    assert n_ar == L + 1 and ar_ms > 0.0 and fwd_ms > 0.0, (fwd_ms, ar_ms, n_ar)
    assert r0["status"] == r1["status"] and np.array_equal(r0["trace"], r1["trace"]), (r0, r1)
    out = O.network_hmc_step(brs, Xs, y.astype(np.float64), 0.1, 0.9, [e.astype(np.float64) for e in eps],
                             [p.astype(np.float64) for p in mom], L, 10.0, 0.3)
    assert r1["status"] == out["status"]
    tr = np.asarray(out["trace"])
    assert np.all(np.abs(r1["trace"][: tr.size] - tr) <= 1e-5 * np.maximum(1.0, np.abs(tr)))
    for b, br in enumerate(brs):
        assert np.array_equal(plain.get_params(b), rccl.get_params(b)), b
        assert norm_rel(rccl.get_params(b), O.param_vec(br.weights, br.biases)) < 1e-5, b
    # library-drawn momenta and uniform (rank 0's draw shared through the f64 all-reduce)
    r0 = plain.network_hmc_step(y, L, bias=0.1, lambda_e=0.9, step_factor=0.3, seed=21)
    r1 = rccl.network_hmc_step(y, L, bias=0.1, lambda_e=0.9, step_factor=0.3, seed=21)
    assert r0["status"] == r1["status"] and np.array_equal(r0["trace"], r1["trace"])
    # a leapfrog session, then the residual exchange on the device (RCCL sum over one rank)
    all_b = list(range(len(specs)))
    for ctx in (plain, rccl):
        ctx.residual_set(y)
        ctx.rebuild_targets(all_b)
        ctx.leapfrog_begin(all_b, 4, 10.0, "izmailov", 0.3, seed=5)
        ctx.leapfrog_steps(4)
        ctx.leapfrog_end()
    d0 = plain.residual_delta()
    plain.exchange_residual_device()
    rccl.exchange_residual_device()
    res0, res1 = plain.residual_get(), rccl.residual_get()
    assert np.array_equal(res0, res1)
    assert np.array_equal(res0, y - d0)
    assert np.any(d0 != 0.0)   # something was accepted: the exchange moved the residual
    # host-residual variant through the RCCL device sum
    assert np.array_equal(plain.exchange_residual(y), rccl.exchange_residual(y))
    plain.close()
    rccl.close()


def _torch_rccl_worker(rank, port, out):
    """torch's own RCCL process group (backend "nccl", as bench.py at N > 1) live in the
    same process as the library's RCCL communicator"""
    import torch
    import torch.distributed as dist
    from bann.distributed import comm_unique_id
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    t = torch.ones(8, device="cuda:0")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    rng, g, specs = _problem(seed=21)
    n, L = g.shape[1], 4
    y = rng.normal(size=n).astype(np.float32)
    eps, mom = _draws(rng, specs, L)
    res = []
    for use_rccl in (False, True):
        ctx = _context(g, specs, range(len(specs)))
        if use_rccl:
            ctx.comm_init_rccl(comm_unique_id(), 1, 0)
            out["info"] = ctx.comm_info()
        r = ctx.network_hmc_step(y, L, bias=0.0, lambda_e=1.0, eps=np.concatenate(eps),
                                 momentum=np.concatenate(mom), u=0.5)
        res.append((r["status"], r["trace"], [ctx.get_params(i) for i in range(len(specs))]))
        ctx.close()
    dist.all_reduce(t)   # torch's communicator still works after the library's
    torch.cuda.synchronize()
    out["torch_sum"] = float(t[0].item())
    out["same"] = bool(res[0][0] == res[1][0] and np.array_equal(res[0][1], res[1][1]) and
                       all(np.array_equal(a, b) for a, b in zip(res[0][2], res[1][2])))
    dist.destroy_process_group()


def test_library_rccl_beside_torch_rccl():
    """bench.py at N > 1 runs torch.distributed over RCCL (backend "nccl") AND the
    library's own RCCL communicator in every rank process: both initialise and
    work side by side (one rank on the one GPU of the box)."""
    import torch.multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_torch_rccl_worker, args=(_free_port(), out), nprocs=1, join=True)
    assert out["info"]["kind"] == "rccl" and out["info"]["backend_ranks"] == 1
    assert out["same"] and out["torch_sum"] == 1.0


@pytest.mark.parametrize("net_err,big", [("1", False), ("0", False), ("1", True), ("0", True)])
def test_network_hmc_fx_only_matches_oracle(monkeypatch, net_err, big):
    """a network of fx branches only (C3's kind): the gradient kernel reads the
    network's output error e = sum f + bias - y itself (DevState::nete,
    BANN_NET_ERR=1, the default) instead of per-branch targets y_b = f_b - e; both
    reproduce the oracle's -H trace, status and parameters"""
    monkeypatch.setenv("BANN_NET_ERR", net_err)
    rng = np.random.default_rng(31)
    # big: C3's branch shape (8 full marker chunks: the full8 kernel) and many tiles per wave
    n = 20000 if big else 1500
    shapes = ([(500, [4, 4, 1])] * 4) if big else [(60, [4, 4, 1]), (100, [4, 4, 1]), (33, [4, 3, 1]), (64, [4, 4, 1])]
    M = sum(m for m, _ in shapes)
    g = O.synthetic_genotypes(rng, n, M)
    specs, off = [], 0
    for m, w in shapes:
        specs.append(dict(snps=np.arange(off, off + m, dtype=np.int32),
                          branch=f32_branch(O.random_branch(rng, m, w, prior="ridge_ard"))))
        off += m
    ctx = _context(g, specs, range(len(specs)))
    assert all(ctx.kernel_path(b) == "fused" for b in range(len(specs)))
    mu, sd = ctx.genotype_stats()
    Xs = [x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]]) for s in specs]
    f = sum(O.predict(s["branch"], X) for s, X in zip(specs, Xs))
    y = (f + rng.normal(scale=0.5, size=n)).astype(np.float32).astype(np.float64)
    L = 8
    for u in (0.3, 0.9):
        eps, mom = _draws(rng, specs, L)
        res = ctx.network_hmc_step(y, L, bias=0.1, lambda_e=2.0, eps=np.concatenate(eps),
                                   momentum=np.concatenate(mom), u=u)
        brs = [s["branch"].copy() for s in specs]
        out = O.network_hmc_step(brs, Xs, y, 0.1, 2.0, [e.astype(np.float64) for e in eps],
                                 [p.astype(np.float64) for p in mom], L, 10.0, u)
        assert res["status"] == out["status"], (res["status"], out["status"], res["trace"], out["trace"])
        tr = np.asarray(out["trace"])
        assert np.all(np.abs(res["trace"][: tr.size] - tr) <= 1e-5 * np.maximum(1.0, np.abs(tr))), (res["trace"], tr)
        for b, br in enumerate(brs):
            assert norm_rel(ctx.get_params(b), O.param_vec(br.weights, br.biases)) < 1e-5, b
        _check_final_targets(ctx, brs, Xs, y, 0.1)
        for s, br in zip(specs, brs):
            s["branch"] = f32_branch(br)
    ctx.close()


@pytest.mark.parametrize("fx_only", [True, False])
def test_common_mode_step_rule(fx_only):
    """bann_set_network_step_rule (default on): before the trajectory one gradient launch
    with output error 1 gives g = J^T 1, and the Izmailov steps become eps_p min(1, t / a_p),
    a_p = eps_p |g_p|, with t the largest histogram candidate (within 2^(1/4) of the exact
    water-filling threshold of oracle.common_mode_steps) keeping lambda_e / n sum min(a, t)^2
    <= tau^2.  The trajectory itself matches the oracle run with the device's step sizes."""
    rng = np.random.default_rng(13)
    n = 1500
    shapes = ([(60, [4, 4, 1], "ridge_ard")] * 8) if fx_only else SHAPES + [(60, [4, 4, 1], "ridge_ard")] * 4
    M = sum(m for m, _, _ in shapes)
    g = O.synthetic_genotypes(rng, n, M)
    specs, off = [], 0
    for m, w, prior in shapes:
        specs.append(dict(snps=np.arange(off, off + m, dtype=np.int32),
                          branch=f32_branch(O.random_branch(rng, m, w, prior=prior))))
        off += m
    ctx = _context(g, specs, range(len(specs)))
    mu, sd = ctx.genotype_stats()
    Xs = [x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]]) for s in specs]
    f = sum(O.predict(s["branch"], X) for s, X in zip(specs, Xs))
    y = (f + rng.normal(scale=0.5, size=n)).astype(np.float32).astype(np.float64)
    L, c, le = 6, 1.0, 2.0
    brs = [s["branch"].copy() for s in specs]
    eps0 = [O.param_vec(*O.izmailov_step_sizes(br, c, L)) for br in brs]
    _, t_exact, a = O.common_mode_steps(brs, Xs, eps0, le, 1.0)
    assert np.isfinite(t_exact)
    mom = [rng.normal(size=s["branch"].num_params).astype(np.float32) for s in specs]
    res = ctx.network_hmc_step(y, L, bias=0.1, lambda_e=le, step_mode="izmailov", step_factor=c,
                               momentum=np.concatenate(mom), u=0.5)
    info = ctx.network_step_rule_info()
    t = info["threshold"]
    assert t_exact * 2 ** -0.25 * (1 - 1e-4) <= t <= t_exact * (1 + 1e-4), (t, t_exact)
    assert 0.0 < info["fraction_scaled"] < 1.0 and info["mode_after"] <= 1.0 + 1e-6
    eps_dev = [ctx.get_step_sizes(b).astype(np.float64) for b in range(len(specs))]
    for e0, ed, x in zip(eps0, eps_dev, a):
        assert norm_rel(ed, e0 * np.minimum(1.0, t / x)) < 1e-5
    out = O.network_hmc_step(brs, Xs, y, 0.1, le, eps_dev, [p.astype(np.float64) for p in mom], L, 10.0, 0.5)
    assert res["status"] == out["status"]
    tr = np.asarray(out["trace"])
    assert np.all(np.abs(res["trace"][: tr.size] - tr) <= 1e-5 * np.maximum(1.0, np.abs(tr)))
    for b, br in enumerate(brs):
        assert norm_rel(ctx.get_params(b), O.param_vec(br.weights, br.biases)) < 1e-5, b
    ctx.set_network_step_rule(False)   # off: the plain Izmailov steps
    ctx.network_hmc_step(y, 2, bias=0.1, lambda_e=le, step_mode="izmailov", step_factor=c, seed=3)
    eps_off = [O.param_vec(*O.izmailov_step_sizes(br, c, 2)) for br in brs]
    for b in range(len(specs)):
        assert norm_rel(ctx.get_step_sizes(b), eps_off[b]) < 2e-7
    ctx.close()


def test_common_mode_rule_frozen():
    """bann_set_network_step_rule(2): the step factors adapted before the last trajectory are
    applied again without recomputing g, so a frozen trajectory's step sizes do not depend on
    the state it starts from (HMC's reversibility; the sampler adapts during burn-in only):
    after an adapted trajectory moved the state, the frozen trajectories take bit for bit the
    adapted step sizes."""
    rng = np.random.default_rng(13)  # test_common_mode_step_rule's fx-only network: the rule scales
    n = 1500
    shapes = [(60, [4, 4, 1], "ridge_ard")] * 8
    M = sum(m for m, _, _ in shapes)
    g = O.synthetic_genotypes(rng, n, M)
    specs, off = [], 0
    for m, w, prior in shapes:
        specs.append(dict(snps=np.arange(off, off + m, dtype=np.int32),
                          branch=f32_branch(O.random_branch(rng, m, w, prior=prior))))
        off += m
    ctx = _context(g, specs, range(len(specs)))
    mu, sd = ctx.genotype_stats()
    Xs = [x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]]) for s in specs]
    y = (sum(O.predict(s["branch"], X) for s, X in zip(specs, Xs))
         + rng.normal(scale=0.5, size=n)).astype(np.float32).astype(np.float64)
    L, c, le = 6, 1.0, 2.0
    ctx.network_hmc_step(y, L, bias=0.1, lambda_e=le, step_mode="izmailov", step_factor=c, seed=5)
    info_a = ctx.network_step_rule_info()
    assert np.isfinite(info_a["threshold"])  # the rule scaled some steps
    eps_a = [ctx.get_step_sizes(b).copy() for b in range(len(specs))]
    ctx.set_network_step_rule("frozen")
    for seed in (6, 7):  # two frozen trajectories from the states the previous ones left
        ctx.network_hmc_step(y, L, bias=0.1, lambda_e=le, step_mode="izmailov", step_factor=c, seed=seed)
        for b in range(len(specs)):
            assert np.array_equal(ctx.get_step_sizes(b), eps_a[b]), b
    ctx.close()


def _fx_network(seed=13, n=1500, nbr=8):
    rng = np.random.default_rng(seed)
    shapes = [(60, [4, 4, 1], "ridge_ard")] * nbr
    M = sum(m for m, _, _ in shapes)
    g = O.synthetic_genotypes(rng, n, M)
    specs, off = [], 0
    for m, w, prior in shapes:
        specs.append(dict(snps=np.arange(off, off + m, dtype=np.int32),
                          branch=f32_branch(O.random_branch(rng, m, w, prior=prior))))
        off += m
    ctx = _context(g, specs, range(len(specs)))
    mu, sd = ctx.genotype_stats()
    Xs = [x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]]) for s in specs]
    y = (sum(O.predict(s["branch"], X) for s, X in zip(specs, Xs))
         + rng.normal(scale=0.5, size=n)).astype(np.float32).astype(np.float64)
    return rng, ctx, specs, Xs, y


def test_common_mode_rule_default_is_state_independent():
    """A caller who never calls bann_set_network_step_rule gets the auto rule (mode 3): the
    first trajectory adapts the common-mode factors (burn-in), every later one applies them
    frozen -- step sizes that depend on the precisions only, not on the trajectory's start
    theta_0, as HMC's detailed balance needs.  Checked by restarting from a different theta_0
    (set_params): the frozen steps are bit for bit the same; the adaptive diagnostic mode (1)
    would change them (so the check can tell the two apart)."""
    rng, ctx, specs, Xs, y = _fx_network()
    L, c, le = 6, 1.0, 2.0
    st = ctx.network_step_rule_state()
    assert st == dict(mode="auto", adapted=0, frozen=False), st
    ctx.network_hmc_step(y, L, bias=0.1, lambda_e=le, step_mode="izmailov", step_factor=c, seed=5)
    assert np.isfinite(ctx.network_step_rule_info()["threshold"])  # the rule scaled some steps
    st = ctx.network_step_rule_state()
    assert st["adapted"] == 1 and st["frozen"], st
    eps_a = [ctx.get_step_sizes(b).copy() for b in range(len(specs))]
    theta_other = []
    for b, s in enumerate(specs):  # a very different start: every parameter scaled and shifted
        th = O.param_vec(s["branch"].weights, s["branch"].biases)
        theta_other.append((1.7 * th + 0.05 * rng.normal(size=th.size)).astype(np.float32))
    for seed in (6, 7):
        for b, th in enumerate(theta_other):
            ctx.set_params(b, th)
        ctx.network_hmc_step(y, L, bias=0.1, lambda_e=le, step_mode="izmailov", step_factor=c, seed=seed)
        for b in range(len(specs)):
            assert np.array_equal(ctx.get_step_sizes(b), eps_a[b]), (seed, b)
    # the diagnostic mode re-adapts from the new theta_0: different steps
    ctx.set_network_step_rule("adaptive")
    for b, th in enumerate(theta_other):
        ctx.set_params(b, th)
    ctx.network_hmc_step(y, L, bias=0.1, lambda_e=le, step_mode="izmailov", step_factor=c, seed=8)
    assert any(not np.array_equal(ctx.get_step_sizes(b), eps_a[b]) for b in range(len(specs)))
    # auto again with K = 2 adapting trajectories
    ctx.set_network_step_rule("auto")
    ctx.set_network_adapt_trajectories(2)
    for k in range(3):
        assert ctx.network_step_rule_state()["frozen"] == (k == 2)
        ctx.network_hmc_step(y, 2, bias=0.1, lambda_e=le, step_mode="izmailov", step_factor=c, seed=20 + k)
    ctx.close()


def test_network_rss_out_on_rejection():
    """bann_network_hmc_step's rss output is the final state's: theta_L when accepted,
    theta_0 (the restored state) when rejected -- checked on a forced early rejection
    against the oracle rss of the starting state."""
    rng, ctx, specs, Xs, y = _fx_network(seed=17, nbr=4)
    ctx.set_network_step_rule("off")
    bias = 0.1
    f0 = sum(O.predict(s["branch"], X) for s, X in zip(specs, Xs))
    rss0 = float(np.sum((y - bias - f0) ** 2))
    eps = np.concatenate([np.full(s["branch"].num_params, 0.5, np.float32) for s in specs])  # absurd steps
    mom = np.concatenate([rng.normal(size=s["branch"].num_params).astype(np.float32) for s in specs])
    res = ctx.network_hmc_step(y, 4, bias=bias, lambda_e=2.0, max_hamiltonian_error=1e-3, eps=eps, momentum=mom,
                               u=0.5)
    assert res["status"] == 2, res["status"]
    assert abs(res["rss"] - rss0) <= 1e-5 * max(1.0, rss0), (res["rss"], rss0)
    for b, s in enumerate(specs):
        assert np.array_equal(ctx.get_params(b), O.param_vec(s["branch"].weights, s["branch"].biases).astype(np.float32))
    ctx.close()


@pytest.mark.parametrize("gsum,passes", [("1", None), ("1", "2"), ("0", None)])
def test_network_group_sum_forward(monkeypatch, gsum, passes):
    """k_forward_gsum (the network forward of 8-chunk fx branches): every step's forward but
    the last sums the branches of an item -- 8 per pass, passes added in order in LDS -- and
    writes one row per item.  Twelve branches (a full pass and a partial one; with
    BANN_NET_GSUM_R=2 both in one item), an odd n (a partial last tile), two trajectories (the
    second starts from current prediction rows, so its step 0 is a group forward too): -H
    trace, status, parameters and the final targets match the oracle, and so does the
    per-branch forward (BANN_NET_GSUM=0)."""
    monkeypatch.setenv("BANN_NET_GSUM", gsum)
    if passes:
        monkeypatch.setenv("BANN_NET_GSUM_R", passes)
    rng = np.random.default_rng(37)
    n = 3001
    shapes = [(500, [4, 4, 1])] * 11 + [(450, [4, 4, 1])]
    M = sum(m for m, _ in shapes)
    g = O.synthetic_genotypes(rng, n, M)
    specs, off = [], 0
    for m, w in shapes:
        specs.append(dict(snps=np.arange(off, off + m, dtype=np.int32),
                          branch=f32_branch(O.random_branch(rng, m, w, prior="ridge_ard"))))
        off += m
    ctx = _context(g, specs, range(len(specs)))
    assert ctx.network_group_rows() == -1
    mu, sd = ctx.genotype_stats()
    Xs = [x_std(g[s["snps"]], mu[s["snps"]], sd[s["snps"]]) for s in specs]
    y = (sum(O.predict(s["branch"], X) for s, X in zip(specs, Xs))
         + rng.normal(scale=0.5, size=n)).astype(np.float32).astype(np.float64)
    L = 6
    for u in (0.3, 0.9):
        eps, mom = _draws(rng, specs, L)
        res = ctx.network_hmc_step(y, L, bias=0.1, lambda_e=2.0, eps=np.concatenate(eps),
                                   momentum=np.concatenate(mom), u=u)
        rows = ctx.network_group_rows()
        if gsum == "0":
            assert rows == 0
        elif passes == "2":
            assert rows == 1   # one item list of 12 branches in two passes
        else:
            assert rows >= 1
        brs = [s["branch"].copy() for s in specs]
        out = O.network_hmc_step(brs, Xs, y, 0.1, 2.0, [e.astype(np.float64) for e in eps],
                                 [p.astype(np.float64) for p in mom], L, 10.0, u)
        assert res["status"] == out["status"], (res["status"], out["status"])
        tr = np.asarray(out["trace"])
        assert np.all(np.abs(res["trace"][: tr.size] - tr) <= 1e-5 * np.maximum(1.0, np.abs(tr))), (res["trace"], tr)
        for b, br in enumerate(brs):
            assert norm_rel(ctx.get_params(b), O.param_vec(br.weights, br.biases)) < 1e-5, b
        _check_final_targets(ctx, brs, Xs, y, 0.1)
        for s, br in zip(specs, brs):
            s["branch"] = f32_branch(br)
    ctx.close()
