"""Multi-GPU sharding for the verify path (one process per GPU).

Signatures are independent, so a batch shards by contiguous signature (or
txn) ranges with no data-path collective.  The only optional
exchange is gathering the per-GPU verdict bitmaps (64M signatures = 8 MB) for
a device-resident consumer; it goes through torch.distributed (RCCL over xGMI
on the GPU box, gloo in the CPU tests).
"""


def shard_bounds(n, rank, world, align=64):
    """Contiguous [lo, hi) of n units for `rank`, boundaries multiples of
    `align` (bitmap words stay whole), every unit in exactly one shard."""
    blocks = (n + align - 1) // align
    lo_b = blocks * rank // world
    hi_b = blocks * (rank + 1) // world
    return min(n, lo_b * align), min(n, hi_b * align)


def gather_bitmap(local_words, n, rank, world, group=None):
    """all_gather the shard bitmaps (int64 tensors, shard_bounds layout) into
    the full ceil(n/64)-word bitmap on every rank."""
    import torch
    import torch.distributed as dist
    words = (n + 63) // 64
    sizes = []
    for r in range(world):
        lo, hi = shard_bounds(n, r, world)
        sizes.append((hi - lo + 63) // 64)
    m = max(sizes) if sizes else 0
    pad = torch.zeros(m, dtype=torch.int64, device=local_words.device)
    pad[:local_words.numel()] = local_words
    outs = [torch.zeros(m, dtype=torch.int64, device=local_words.device) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    full = torch.cat([o[:s] for o, s in zip(outs, sizes)])
    assert full.numel() == words
    return full


def max_over_ranks(x, device=None, group=None):
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
