"""Data parallelism for the RealNVP step: one process per GPU, sample sharding,
one exchange (gradient average) per optimizer step.

The path shards by sample: rank r trains on its own batch slice, BatchNorm
statistics stay local (= the reference's batch-64 semantics per shard), and
the flat gradient arena is averaged with all-reduce in fixed-size buckets
(RCCL over xGMI on MI355X; gloo on CPU for tests).
"""
import torch
import torch.distributed as dist


def bucket_ranges(n, bucket_elems):
    """[start, end) ranges covering [0, n) in buckets of bucket_elems."""
    b = max(1, int(bucket_elems))
    return [(i, min(n, i + b)) for i in range(0, n, b)]


def bucket_schedule(blocks, bucket_elems, n_total):
    """Gradient buckets of the flat arena in the order backward finishes them.

    blocks: (offset, numel) of each coupling's gradient block, in the order
    the backward visits the couplings (descending arena offset: the deep
    scales, which hold most parameters, finish first).  Returns a list of
    (start, end, k): elements [start, end) are final once the k-th block of
    that order has run, so their all-reduce can start then.  Buckets cover
    [0, n_total) exactly once (n_total includes the arena's tail padding,
    which goes with the first bucket)."""
    b = max(1, int(bucket_elems))
    out = []
    hi = int(n_total)
    lo = hi
    for k, (off, n) in enumerate(blocks):
        off, n = int(off), int(n)
        # the first block may end short of n_total (padding); the rest must tile
        if (k == 0 and not (0 <= hi - (off + n) < 64)) or (k > 0 and off + n != lo):
            raise ValueError("gradient blocks must tile the arena downwards in backward order")
        lo = off
        if hi - lo >= b:
            out.append((lo, hi, k))
            hi = lo
    if lo != 0:
        raise ValueError("gradient blocks do not reach offset 0")
    if hi > lo:
        out.append((lo, hi, len(blocks) - 1))
    return out


def average_slice(flat, lo, hi, group=None, buf=None):
    """Average flat[lo:hi) across the group in place (one bucket of the
    trainer's overlapped all-reduce).  buf: an optional bf16 arena the
    bucket is reduced through (half the bytes on the wire)."""
    world = dist.get_world_size(group)
    g = flat[lo:hi]
    if buf is not None:
        b = buf[lo:hi]
        b.copy_(g)
        dist.all_reduce(b, op=dist.ReduceOp.SUM, group=group)
        g.copy_(b)
    else:
        dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group)
    g.mul_(1.0 / world)
    return g


def allreduce_average(flat, group=None, bucket_elems=16 << 20):
    """In-place average of a flat tensor across the group, bucket by bucket."""
    world = dist.get_world_size(group)
    if world == 1:
        return flat
    avg = getattr(dist.ReduceOp, "AVG", None)
    use_avg = avg is not None and dist.get_backend(group) == "nccl"
    for s, e in bucket_ranges(flat.numel(), bucket_elems):
        if use_avg:
            dist.all_reduce(flat[s:e], op=avg, group=group)
        else:
            dist.all_reduce(flat[s:e], op=dist.ReduceOp.SUM, group=group)
            flat[s:e].div_(world)
    return flat


def max_over_ranks(value, device, group=None):
    """max of a python float over ranks (the bench's timing rule)."""
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def mean_over_ranks(value, device, group=None):
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t /= dist.get_world_size(group)
    return float(t.item())


def rank_seed(base, rank):
    """Per-rank data seed: every rank draws a different batch (weak scaling)."""
    return int(base) * 1000003 + int(rank)
