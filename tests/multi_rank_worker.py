"""One rank of the sharded verify (tests/test_gpu_multi.py launches 2 of
them as fresh processes; gloo carries the bitmap gather, every rank holds its
own verify context on GPU 0).

Each rank builds the same seeded C2-mix batch (GPU signer + C2 mutation),
verifies its shard_bounds slice through the C ABI (fd_ed25519_hip_verify_dev
on its own context and stream) and all-gathers the verdict bitmap
(firedancer_amd.shard.gather_bitmap).  Rank 0 then checks the gathered
bitmap against a single-process whole-batch pass, and that pass's codes
against the CPU oracle on a random 8K sample (test infrastructure only).
Writes a JSON verdict to argv[2].

usage: python tests/multi_rank_worker.py <n_sigs> <out.json>   (RANK, WORLD_SIZE,
       MASTER_ADDR, MASTER_PORT in the environment)
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    n, out_path = int(sys.argv[1]), sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from firedancer_amd import Verifier
    from firedancer_amd.shard import gather_bitmap, max_over_ranks, shard_bounds
    from firedancer_amd.workload import make_batch_gpu

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    gen = Verifier(device=0, chunk_sigs=1 << 20)
    b = make_batch_gpu(gen, n, msg_sz=64, seed=0xc5c5, mix="c2")          # identical on every rank
    torch.cuda.synchronize()

    lo, hi = shard_bounds(n, rank, world)
    m = hi - lo
    v = Verifier(device=0, chunk_sigs=1 << 20)                             # this rank's context
    codes = torch.full((max(m, 1),), 9, dtype=torch.int8, device=dev)
    words = torch.zeros(max((m + 63) // 64, 1), dtype=torch.int64, device=dev)
    t0 = time.perf_counter()
    v.verify_dev(m, b.sigs[lo:hi], b.pubs[lo:hi], b.pool, b.msg_off[lo:hi], b.msg_sz[lo:hi], codes, words)
    torch.cuda.synchronize()
    dt = max_over_ranks(time.perf_counter() - t0)
    full = gather_bitmap(words[:(m + 63) // 64].cpu(), n, rank, world)      # gloo: host tensors

    res = {"rank": rank, "lo": lo, "hi": hi, "shard_ms_max": dt * 1e3}
    if rank == 0:
        whole_codes = torch.full((n,), 9, dtype=torch.int8, device=dev)
        whole_bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
        w = Verifier(device=0, chunk_sigs=1 << 20)
        w.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, whole_codes, whole_bm)
        torch.cuda.synchronize()
        c = whole_codes.cpu().numpy()
        res["bitmap_equal"] = bool(torch.equal(full, whole_bm.cpu()))
        bits = np.unpackbits(whole_bm.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
        res["bitmap_is_codes"] = bool(np.array_equal(bits, c == 0))
        res["accept"] = float((c == 0).mean())
        res["codes_set"] = bool(np.isin(c, (0, -1, -2, -3)).all())
        import oracle_lib as O
        idx = np.sort(np.random.default_rng(5).choice(n, 8192, replace=False))
        ti = torch.from_numpy(idx).to(dev)
        sigs = b.sigs[ti].cpu().numpy(); pubs = b.pubs[ti].cpu().numpy()
        moff = b.msg_off[ti].cpu().numpy().view(np.uint32); msz = b.msg_sz[ti].cpu().numpy().view(np.uint32)
        pool = b.pool.cpu().numpy()
        exp = O.verify_many(sigs, pubs, pool, moff, msz)
        res["oracle_sample_equal"] = bool(np.array_equal(c[idx], exp))
        w.close()
    v.close(); gen.close()
    dist.barrier()
    dist.destroy_process_group()
    with open(out_path, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
