"""World-size-2 data-parallel logic on CPU (gloo): bucketed gradient averaging,
max-over-ranks timing, per-rank batches."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    from realnvp_hip import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 1000003
        g = torch.arange(n, dtype=torch.float32) * (rank + 1)
        D.allreduce_average(g, bucket_elems=65536)
        expect = torch.arange(n, dtype=torch.float32) * (sum(r + 1 for r in range(world)) / world)
        ok_avg = bool(torch.allclose(g, expect))
        t = D.max_over_ranks(1.0 + rank, "cpu")
        m = D.mean_over_ranks(float(rank), "cpu")
        seeds = [D.rank_seed(7, r) for r in range(world)]
        out[rank] = (ok_avg, t, m, len(set(seeds)) == world)
    finally:
        dist.destroy_process_group()


def test_bucket_ranges_cover_exactly():
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    from realnvp_hip.dist import bucket_ranges
    for n, b in ((10, 3), (12, 4), (1, 100), (120090296, 16 << 20)):
        r = bucket_ranges(n, b)
        assert r[0][0] == 0 and r[-1][1] == n
        assert all(r[i][1] == r[i + 1][0] for i in range(len(r) - 1))


def test_gloo_world2_average_and_timing():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    for r in range(world):
        ok_avg, t, m, distinct = out[r]
        assert ok_avg
        assert t == float(world)          # max over ranks
        assert m == sum(range(world)) / world
        assert distinct


def _bucket_worker(rank, world, port, out):
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    import flow_realnvp
    import utils
    from realnvp_hip import dist as D
    from realnvp_hip.trainer import arena_blocks, bucket_plan
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        prior = torch.distributions.Normal(torch.tensor(0.0), torch.tensor(1.0))
        model = flow_realnvp.RealNVP(3, 32, prior, utils.Hyperparameters(8, 1, True, True, True, True))
        n = sum(p.numel() for p in model.parameters())
        n_pad = (n + 3) // 4 * 4
        blocks = arena_blocks(model)
        plan = bucket_plan(model, 16384, n_pad)
        # the trainer's grad arena: rank-dependent values; reduce bucket by bucket
        # in the order backward would issue them (bf16 wire format on every other bucket)
        g = torch.arange(n_pad, dtype=torch.float32).remainder_(997.0) * (rank + 1)
        buf = torch.empty(n_pad, dtype=torch.bfloat16)
        for i, (lo, hi, k) in enumerate(plan):
            D.average_slice(g, lo, hi, buf=buf if i % 2 else None)
        expect = torch.arange(n_pad, dtype=torch.float32).remainder_(997.0) * (sum(r + 1 for r in range(world)) / world)
        bf = torch.zeros(n_pad, dtype=torch.bool)
        for i, (lo, hi, k) in enumerate(plan):
            if i % 2:
                bf[lo:hi] = True
        ok32 = bool(torch.equal(g[~bf], expect[~bf]))
        ok16 = bool(torch.allclose(g[bf], expect[bf], rtol=1e-2))
        out[rank] = (ok32, ok16, plan, blocks, n_pad)
    finally:
        dist.destroy_process_group()


def test_gloo_world2_bucket_schedule_over_arena():
    """The trainer's overlapped all-reduce schedule over the real parameter
    arena of a RealNVP: buckets tile the arena once, each is issued only after
    every coupling whose parameters it holds has finished its backward, and
    reducing bucket by bucket (fp32 or bf16 wire) averages the ranks."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0
    ok32, ok16, plan, blocks, n_pad = out[0]
    assert ok32 and ok16 and out[1][0] and out[1][1]
    assert out[1][2] == plan
    assert len(plan) > 4
    # tiling: descending, contiguous, exact cover
    assert plan[0][1] == n_pad and plan[-1][0] == 0
    assert all(plan[i][0] == plan[i + 1][1] for i in range(len(plan) - 1))
    bwd = list(reversed(blocks))      # backward visits couplings in reverse
    for lo, hi, k in plan:
        # every parameter in [lo, hi) belongs to a coupling at backward position <= k
        first_ready = bwd[k][0]
        assert lo >= first_ready
        assert k == 0 or lo < bwd[k - 1][0]
