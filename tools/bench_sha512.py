"""Batched SHA-512 throughput on one GPU (fd_sha512_hip_batch_dev), messages
resident in HBM, one kernel launch per batch, timed with HIP events on the
launch stream.  Prints one JSON line per message size.

    python tools/bench_sha512.py [--n 1048576] [--sizes 64,1232,4096] [--reps 10]

Reported: messages/s, message GB/s, 128-byte blocks/s, and the blocks' share
of the VALU issue budget at the reference cost SURVEY.md 8(d) uses for one
block (4 900 32-bit operations; peak 39.3e12 lane-operations/s).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--sizes", default="64,1232,4096")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import hashlib

    import numpy as np
    import torch

    from firedancer_amd import Verifier
    from firedancer_amd.ed25519 import CTX_STREAM
    from firedancer_amd.sha512 import sha512_batch_dev
    dev = torch.device("cuda", 0)
    v = Verifier(device=0, chunk_sigs=1 << 16)
    s = torch.cuda.ExternalStream(v.stream, device=dev)
    for sz in (int(x) for x in a.sizes.split(",")):
        n = a.n
        stride = (sz + 15) // 16 * 16
        g = torch.Generator(device=dev).manual_seed(sz)
        pool = torch.randint(0, 256, (n * stride + 16,), dtype=torch.uint8, device=dev, generator=g)
        off = (torch.arange(n, device=dev, dtype=torch.int64) * stride).to(torch.int32)
        msz = torch.full((n,), sz, dtype=torch.int32, device=dev)
        out = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        sha512_batch_dev(v, n, pool, off, msz, out, stream=CTX_STREAM)     # warm
        v.sync()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            sha512_batch_dev(v, n, pool, off, msz, out, stream=CTX_STREAM)
        e1.record(s)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        idx = np.random.default_rng(sz).choice(n, 64, replace=False)
        p = pool.cpu().numpy(); o = out.cpu().numpy()
        ok = all(hashlib.sha512(p[i * stride:i * stride + sz].tobytes()).digest() == o[i].tobytes() for i in idx)
        blocks = (sz + 17 + 127) // 128
        bps = n * blocks / (ms * 1e-3)
        print(json.dumps({"what": "fd_sha512_hip_batch_dev", "msg_bytes": sz, "messages": n, "ms_per_launch": round(ms, 4),
                          "messages_per_s": round(n / (ms * 1e-3), 1), "msg_GBps": round(n * sz / (ms * 1e-3) / 1e9, 2),
                          "blocks_per_s": round(bps, 1), "ref_block_ops_vs_int32_peak": round(bps * 4900 / 39.3e12, 4),
                          "sample_equal_hashlib": ok}), flush=True)
        del pool, off, msz, out
    v.close()


if __name__ == "__main__":
    main()
