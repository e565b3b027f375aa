"""CPU: the N>1 path (signature shards + bitmap gather + max-over-ranks) on a
world_size-2 gloo group."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from firedancer_amd.shard import gather_bitmap, max_over_ranks, shard_bounds


def test_shard_bounds_partition():
    for n in (0, 1, 63, 64, 65, 1000, 1 << 20, (1 << 26) + 5):
        for world in (1, 2, 3, 4, 8):
            cover = []
            for r in range(world):
                lo, hi = shard_bounds(n, r, world)
                assert lo % 64 == 0 and (hi % 64 == 0 or hi == n)
                cover.append((lo, hi))
            assert cover[0][0] == 0 and cover[-1][1] == n
            for (a, b), (c, d) in zip(cover, cover[1:]):
                assert b == c


def _worker(rank, world, port, n, ret):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(42)
    codes = rng.integers(-3, 1, n).astype(np.int8)           # same global "verdicts" on every rank
    lo, hi = shard_bounds(n, rank, world)
    mine = codes[lo:hi] == 0                                   # this rank's shard verdicts
    bits = np.packbits(mine, bitorder="little")
    bits = np.concatenate([bits, np.zeros((-bits.size) % 8, np.uint8)]).view(np.int64)
    full = gather_bitmap(torch.from_numpy(bits.copy()), n, rank, world)
    got = np.unpackbits(full.numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
    ok = bool(np.array_equal(got, codes == 0))
    t = max_over_ranks(1.0 + rank)
    ret[rank] = (ok, t)
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [1000, 4096 + 17])
def test_gloo_world2_bitmap_gather(n):
    world = 2
    mgr = mp.Manager()
    ret = mgr.dict()
    port = 29500 + (os.getpid() % 1000)
    mp.spawn(_worker, args=(world, port, n, ret), nprocs=world, join=True)
    assert all(ret[r][0] for r in range(world))
    assert all(ret[r][1] == float(world) for r in range(world))


def test_bench_c5_shards_cover_2p26():
    """bench.py's C5 shard arithmetic (c5_shard) covers 2^26 signatures
    exactly, contiguously and disjointly at world 1/2/4/8, with bitmap-word
    aligned boundaries and per-rank shards the 2^20-signature chunking of a
    context splits without remainder."""
    import bench
    for world in (1, 2, 4, 8):
        spans = [bench.c5_shard(None, r, world) for r in range(world)]
        assert all(t == 1 << 26 for t, _, _ in spans)
        assert spans[0][1] == 0 and spans[-1][2] == 1 << 26
        for (_, _, hi), (_, lo, _) in zip(spans, spans[1:]):
            assert hi == lo
        sizes = [hi - lo for _, lo, hi in spans]
        assert sum(sizes) == 1 << 26 and len(set(sizes)) == 1
        assert all(s % 64 == 0 and s % (1 << 20) == 0 for s in sizes)
    t, lo, hi = bench.c5_shard(1 << 21, 1, 2)               # --sigs per rank (the gloo rehearsal)
    assert (t, lo, hi) == (1 << 22, 1 << 21, 1 << 22)


def test_c5_global_set_ranges_are_slices():
    """config 5's global set (workload.range_inputs): any block-aligned or
    unaligned range [lo, hi) is exactly that slice of the whole set, so a
    rank that generates only its shard verifies the whole-set records."""
    import numpy as np
    from firedancer_amd.workload import range_inputs
    blk, total = 1 << 10, 1 << 13
    prv, pool, moff, msz = range_inputs(0, total, block=blk)
    assert prv.shape == (total, 32) and pool.size == 64 * total + 16
    for lo, hi in ((0, blk), (blk, 3 * blk), (5 * blk, total), (100, 4000), (2047, 2049)):
        p2, q2, o2, s2 = range_inputs(lo, hi, block=blk)
        assert np.array_equal(p2, prv[lo:hi])
        assert np.array_equal(q2[:-16], pool[64 * lo:64 * hi]) and not q2[-16:].any()
        assert np.array_equal(o2, moff[:hi - lo]) and (s2 == 64).all()
    # different blocks draw different keys
    assert not np.array_equal(prv[:blk], prv[blk:2 * blk])
