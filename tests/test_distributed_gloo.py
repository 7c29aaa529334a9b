"""Multi-rank path on CPU (gloo, world_size 2), driven through the library's C ABI:
bann_shard_branches balances the branch ranges, and bann_residual_update_host --
the exchange step bann_exchange_residual runs for a callback communicator --
sums the ranks' residual changes through a gloo all-reduce callback
(bann.distributed.TorchAllreduce); every rank ends with the single-rank residual.

The per-branch predictions come from the oracle (test infrastructure, there is
no GPU here); what is under test is the library's sharding and exchange code."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bann_oracle as O
from bann.distributed import TorchAllreduce, residual_update, shard_ranges


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem():
    rng = np.random.default_rng(3)
    n, B = 200, 7
    ms = [30, 10, 25, 40, 5, 30, 12]
    M = sum(ms)
    g = O.synthetic_genotypes(rng, n, M)
    mu, sd = O.bed_col_stats(g)
    X = ((g.T - mu) / sd)
    offs = np.concatenate([[0], np.cumsum(ms)])
    brs = [O.random_branch(rng, ms[b], [3, 2, 1]) for b in range(B)]
    news = [O.random_branch(rng, ms[b], [3, 2, 1]) for b in range(B)]
    accepted = [True, False, True, True, False, True, True]
    y = rng.normal(size=n)
    return n, ms, offs, X, brs, news, accepted, y


def _local_delta(rank, world):
    n, ms, offs, X, brs, news, accepted, y = _problem()
    lo, hi = shard_ranges(ms, world)[rank]
    d = np.zeros(n)
    for b in range(lo, hi):
        if accepted[b]:
            Xb = X[:, offs[b]:offs[b + 1]]
            d += O.predict(news[b], Xb) - O.predict(brs[b], Xb)
    return d.astype(np.float32)


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, ms, offs, X, brs, news, accepted, y = _problem()
    residual = (y - sum(O.predict(brs[b], X[:, offs[b]:offs[b + 1]]) for b in range(len(ms)))).astype(np.float32)
    res = residual_update(residual, _local_delta(rank, world), TorchAllreduce(dist))
    out[rank] = res.copy()
    dist.destroy_process_group()


def test_shard_ranges_balanced():
    r = shard_ranges([500] * 1000, 8)
    assert r[0] == (0, 125) and r[-1] == (875, 1000)
    assert all(b - a == 125 for a, b in r)
    r = shard_ranges([1, 1, 10, 1, 1, 10], 2)
    assert r[0][0] == 0 and r[-1][1] == 6 and r[0][1] == r[1][0]
    # one dominant branch never leaves a rank empty
    r = shard_ranges([1000, 1, 1, 1], 4)
    assert r == [(0, 1), (1, 2), (2, 3), (3, 4)]
    with pytest.raises(ValueError):   # more ranks than branches
        shard_ranges([5, 5], 3)


def test_sharded_residual_update_matches_single_rank():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    n, ms, offs, X, brs, news, accepted, y = _problem()
    ref = residual_update((y - sum(O.predict(brs[b], X[:, offs[b]:offs[b + 1]]) for b in range(len(ms)))
                           ).astype(np.float32), _local_delta(0, 1), None)
    for r in range(world):
        assert np.allclose(out[r], ref, rtol=0, atol=1e-5)
    assert np.array_equal(out[0], out[1])
