#!/usr/bin/env python3
"""Per-call latency of the link-compatible drop-in entry points on the GPU
box: fd_ed25519_verify and fd_ed25519_verify_batch_single_msg (batch_sz 1, 12,
16), called through the C ABI (ctypes) exactly as a reference caller would,
one call at a time.  Prints one JSON object (p50/p99/mean in microseconds).

usage: python tools/bench_latency.py [calls]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    import torch
    from firedancer_amd import Verifier
    from firedancer_amd.build import LIB
    from firedancer_amd.workload import make_batch_gpu
    v = Verifier(device=0, chunk_sigs=4096)
    msg_sz = 200
    b = make_batch_gpu(v, 16, msg_sz=msg_sz, seed=5, mix="c1", shared_msg=True)
    torch.cuda.synchronize()
    sigs = b.sigs.cpu().numpy().tobytes(); pubs = b.pubs.cpu().numpy().tobytes()
    msg = b.pool[:msg_sz].cpu().numpy().tobytes()
    v.close()
    L = ctypes.CDLL(os.environ.get("FD_ED25519_HIP_LIB") or LIB)   # a build variant, as firedancer_amd.ed25519 loads it
    c = ctypes
    L.fd_ed25519_verify.argtypes = [c.c_char_p, c.c_ulong, c.c_char_p, c.c_char_p, c.c_void_p]
    L.fd_ed25519_verify_batch_single_msg.argtypes = [c.c_char_p, c.c_ulong, c.c_char_p, c.c_char_p, c.c_void_p,
                                                     c.c_ubyte]
    out = {"calls": calls, "msg_sz": msg_sz, "unit": "us"}

    def measure(fn):
        for _ in range(50):
            assert fn() == 0
        t = np.empty(calls)
        for i in range(calls):
            t0 = time.perf_counter()
            r = fn()
            t[i] = time.perf_counter() - t0
            assert r == 0
        t *= 1e6
        return {"p50": round(float(np.percentile(t, 50)), 1), "p99": round(float(np.percentile(t, 99)), 1),
                "mean": round(float(t.mean()), 1), "min": round(float(t.min()), 1)}

    out["fd_ed25519_verify"] = measure(lambda: L.fd_ed25519_verify(msg, msg_sz, sigs[:64], pubs[:32], None))
    for n in (1, 12, 16):
        out[f"batch_single_msg_{n}"] = measure(
            lambda n=n: L.fd_ed25519_verify_batch_single_msg(msg, msg_sz, sigs[:64 * n], pubs[:32 * n], None, n))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
