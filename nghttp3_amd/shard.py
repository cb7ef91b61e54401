"""Node-level sharding of Huffman batches.

Strings (and, with the dynamic table off, whole header blocks) are
independent, so a batch splits into contiguous string ranges with no
data-path exchange: each rank receives its shard by its own H2D copy and
decodes it alone.  Collectives (RCCL over xGMI on MI355X, gloo on CPU) carry
only the report: max of the per-rank time, sums of bytes / errors, and the
exclusive prefix of per-rank output sizes that places each shard's output in
a global layout.
"""
from __future__ import annotations

import numpy as np


def shard_seed(seed: int, rank: int) -> int:
    """Weak-scaling synthetic input: rank r generates batch seed + r (rank 0
    keeps the configuration's own seed so its digests stay comparable)."""
    return seed + rank


def split_by_bytes(lengths, world: int):
    """Contiguous string ranges [(begin, end)] with near-equal byte totals.

    Boundaries are placed at the first string whose exclusive byte prefix
    reaches k * total / world (k = 1 .. world-1).
    """
    ln = np.asarray(lengths, dtype=np.uint64)
    n = ln.size
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(world - 1, 0)
    prefix = np.zeros(n + 1, dtype=np.uint64)
    prefix[1:] = np.cumsum(ln)
    total = int(prefix[-1])
    cuts = [0]
    for k in range(1, world):
        target = (total * k) // world
        cuts.append(int(np.searchsorted(prefix[:-1], target, side="left")))
    cuts.append(n)
    cuts = [min(max(c, 0), n) for c in cuts]
    for i in range(1, len(cuts)):
        cuts[i] = max(cuts[i], cuts[i - 1])
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


def reduce_report(local: dict, dist=None, device=None) -> dict:
    """All-reduce a per-rank report: keys ending in '_max' take the max,
    everything else is summed.  Without an initialised process group the
    local report is returned unchanged."""
    keys = sorted(local)
    if dist is None or not dist.is_available() or not dist.is_initialized():
        return dict(local)
    import torch
    maxk = [k for k in keys if k.endswith("_max")]
    sumk = [k for k in keys if not k.endswith("_max")]
    out = {}
    for group, op in ((maxk, dist.ReduceOp.MAX), (sumk, dist.ReduceOp.SUM)):
        if not group:
            continue
        t = torch.tensor([float(local[k]) for k in group], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=op)
        out.update({k: float(v) for k, v in zip(group, t.tolist())})
    return out


def output_offsets(local_bytes: int, dist=None, device=None) -> int:
    """Exclusive prefix of per-rank output sizes (all-gather of one u64 per
    rank): where this rank's shard starts in a node-global output layout."""
    if dist is None or not dist.is_available() or not dist.is_initialized():
        return 0
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    t = torch.tensor([int(local_bytes)], dtype=torch.int64, device=device)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return int(sum(int(p.item()) for p in parts[:rank]))


def block_range(rank: int, world: int, nblocks: int):
    """Rank's contiguous range of nblocks header blocks, [lo, hi), by block
    count (block_range_by_bytes is what config 4 uses)."""
    return rank * nblocks // world, (rank + 1) * nblocks // world


def block_range_by_bytes(rank: int, world: int, block_lens):
    """Config 4: rank's contiguous range of header blocks, [lo, hi), cut at
    near-equal block bytes (split_by_bytes over the blocks' lengths: real
    traffic mixes short and long sections, so a cut by count would leave
    ranks unequal work).  Blocks at dynamic table 0 are independent, so ranks
    share nothing but the report (strong scaling over a fixed corpus).

    A cut by bytes can leave a rank no block (one block larger than a
    rank's share); every rank then takes the cut by count instead, so no
    rank has an empty range while world <= len(block_lens)."""
    ranges = split_by_bytes(block_lens, world)
    n = len(block_lens)
    if world <= n and any(b == e for b, e in ranges):
        return block_range(rank, world, n)
    return ranges[rank]
