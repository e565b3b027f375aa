"""Time the device half-size reduction alone (fd_ed25519_hip_test_halfsize:
sc_halfsize on n hashed scalars, one lane each) against a verify launch of
the same size, HIP events on the context stream."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import hashlib

    import numpy as np
    import torch

    from firedancer_amd import Verifier
    from firedancer_amd.ed25519 import CTX_STREAM
    n = 1 << 20
    dev = torch.device("cuda", 0)
    v = Verifier(device=0, chunk_sigs=n)
    rng = np.random.default_rng(5)
    # scalars k < L: SHA-512 of random bytes reduced mod L
    L = 2**252 + 27742317777372353535851937790883648493
    ks = [int.from_bytes(hashlib.sha512(rng.bytes(16)).digest(), "little") % L for _ in range(4096)]
    kb = np.frombuffer(b"".join(k.to_bytes(32, "little") for k in ks), np.uint8)
    k = torch.from_numpy(np.tile(kb, n // 4096).view(np.int32)).to(dev)
    out = torch.empty(18 * n, dtype=torch.int32, device=dev)
    s = torch.cuda.ExternalStream(v.stream, device=dev)
    torch.cuda.synchronize()
    v.test_halfsize(n, k, out, stream=CTX_STREAM)
    v.sync()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(5):
        v.test_halfsize(n, k, out, stream=CTX_STREAM)
    e1.record(s)
    e1.synchronize()
    print(json.dumps({"what": "sc_halfsize alone, 2^20 scalars, 64-thread workgroups",
                      "ms_per_launch": round(e0.elapsed_time(e1) / 5, 4)}))


if __name__ == "__main__":
    main()
