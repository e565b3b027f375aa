#!/usr/bin/env python3
"""Call latency and throughput of fd_ed25519_hip_verify_dev against batch
size, inputs resident in HBM (GPU box).  For each n, a C2-mix batch of n
signatures (GPU-signed, 64-B messages) is verified `calls` times, one call at
a time with a stream sync after each (a caller waiting for its verdicts):
p50 / p99 wall time per call and n / p50 as verifies/s.  Each n up to 256
runs twice: on k_verify_lat (one workgroup per signature; <= 32 race one
copy per XCD; set_small_batch(256)) and on k_verify_prep + k_verify_dsm
(set_small_batch(0), keys "<n>_bulk").  The crossover sets the default
small-batch limit (32).

usage: python tools/bench_batch_latency.py [calls]   -> one JSON line
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    import torch
    from firedancer_amd import Verifier
    from firedancer_amd.ed25519 import CTX_STREAM
    from firedancer_amd.workload import make_batch_gpu
    sizes = [1, 2, 4, 8, 16, 32, 64, 256, 1024, 4096, 16384, 65536, 262144]
    v = Verifier(device=0, chunk_sigs=1 << 18)
    b = make_batch_gpu(v, max(sizes), msg_sz=64, seed=11, mix="c2")
    torch.cuda.synchronize()
    codes = torch.zeros(max(sizes), dtype=torch.int8, device=b.dev)
    out = {"calls": calls, "msg_sz": 64, "unit": "us", "inputs": "HBM-resident, C2 mix", "sizes": {}}
    runs = [(n, 256) for n in sizes] + [(n, 0) for n in sizes if n <= 256]   # (n, small-batch limit)
    for n, lim in runs:
        v.set_small_batch(lim)
        k = calls if n <= 65536 else max(10, calls // 10)

        def one():
            v.verify_dev(n, b.sigs[:n], b.pubs[:n], b.pool, b.msg_off[:n], b.msg_sz[:n], codes[:n], stream=CTX_STREAM)
            v.sync()
        for _ in range(5):
            one()
        t = np.empty(k)
        for i in range(k):
            t0 = time.perf_counter()
            one()
            t[i] = time.perf_counter() - t0
        t *= 1e6
        p50 = float(np.percentile(t, 50))
        lat = n <= lim
        key = str(n) if lim else f"{n}_bulk"
        out["sizes"][key] = {"p50_us": round(p50, 1), "p99_us": round(float(np.percentile(t, 99)), 1),
                             "verifies_per_s": round(n / (p50 * 1e-6), 1),
                             "path": "k_verify_lat" + (" x8 copies" if n <= 32 else "") if lat
                             else "k_verify_prep + k_verify_dsm"}
        print(key, out["sizes"][key], file=sys.stderr)
    v.set_small_batch(32)
    v.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
