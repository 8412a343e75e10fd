"""Codeword sharding across GPUs.

Codewords are independent and H is read-only, so a batch splits into
contiguous per-rank shards with no collective on the data path.  Each rank
regenerates its own inputs from (seed, first codeword index), decodes, and
only three counters (bit errors, frame errors, frames) plus the elapsed time
are reduced at the end -- the reference has no distributed layer at all
(no MPI / NCCL anywhere).
"""


def shard_range(rank, world, total):
    """[first, first + count) of `total` codewords owned by `rank` (contiguous, balanced)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def reduce_results(elapsed_s, bit_errors, frame_errors, frames, device=None):
    """(max elapsed, sum errors, sum frame errors, sum frames) over the default
    process group (any backend); identity when torch.distributed is not initialised."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    c = torch.tensor([bit_errors, frame_errors, frames], dtype=torch.int64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
    be, fe, fr = c.tolist()
    return float(t.item()), int(be), int(fe), int(fr)
