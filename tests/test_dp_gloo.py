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
