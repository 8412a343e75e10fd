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


def mixed_layout(rank, world, batch, n_codes):
    """configs[4] (mixed-rate batches) across ranks.  Rank `rank` owns the
    contiguous global codewords [rank * batch, (rank + 1) * batch); global
    codeword g has rate g % n_codes.  Returns (ids, noise_first):

    * ids[i]: the rate of the rank's i-th codeword;
    * noise_first[c]: the channel generator's first codeword index for the
      rank's rate-c sub-batch (its j-th rate-c codeword draws the noise of
      index noise_first[c] + j): c * batch * world + the number of rate-c
      codewords before the rank's first one.

    Every (rate, global codeword) pair gets its own noise index, so ranks never
    draw the same noise (r05 used first_cw + c * batch, which made rank r's
    rate c and rank r + 1's rate c - 1 share their noise), and an N-rank job
    decodes exactly the codewords of one process with batch * world."""
    import numpy as np
    first, count = shard_range(rank, world, batch * world)
    assert count == batch
    ids = ((first + np.arange(batch)) % n_codes).astype(np.int32)
    noise_first = [c * batch * world + max(0, (first - c + n_codes - 1) // n_codes) for c in range(n_codes)]
    return ids, noise_first


def reduce_sums(values, device=None):
    """Element-wise sum of a list of numbers over the default process group
    (float64; identity without torch.distributed)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()
