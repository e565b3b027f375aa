#!/usr/bin/env python3
"""FETCH_SIZE calibration for the prep kernel's message-read pattern
(MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for 16-B-per-lane
streaming reads, where it reports half the bytes).  Hashes 2^20 distinct
messages of 256 B (256 MiB, each read exactly once) through the device hash
test hook, whose two launches are the per-lane dword-load path and the
wave-cooperative LDS-staged path k_verify_prep uses; run under
rocprofv3 --pmc FETCH_SIZE to read the counter against the known bytes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from firedancer_amd import Verifier  # noqa: E402


def main():
    n, msz = 1 << 20, 256
    v = Verifier(device=0, chunk_sigs=4096)
    dev = torch.device("cuda", 0)
    pool = torch.randint(0, 256, (n * msz + 16,), dtype=torch.uint8, device=dev)
    off = torch.arange(n, dtype=torch.int32, device=dev) * msz
    sz = torch.full((n,), msz, dtype=torch.int32, device=dev)
    out = torch.empty((2 * n, 64), dtype=torch.uint8, device=dev)
    for _ in range(2):
        v.test_sha512(n, pool, off, sz, out)
    torch.cuda.synchronize()
    assert torch.equal(out[:n], out[n:])
    print(f"{n} messages x {msz} B = {n * msz} bytes read per launch")


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def records():
    """Second pattern: k_verify_prep on 2^20 records with empty messages, so it
    reads only sig (64 B), pub (32 B) and msg_off/msg_sz (8 B) per record
    (104 MiB... 104 B x 2^20), one 16-B load per lane per piece at a 64-B /
    32-B record stride."""
    from firedancer_amd.workload import make_batch_gpu
    n = 1 << 20
    v = Verifier(device=0, chunk_sigs=n)
    b = make_batch_gpu(v, n, msg_sz=0, seed=3, mix="c1")
    codes = torch.empty(n, dtype=torch.int8, device="cuda:0")
    for _ in range(2):
        v.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes)
    torch.cuda.synchronize()
    print(f"{n} records x 104 B = {n * 104} bytes read per k_verify_prep launch")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "records":
    records()
