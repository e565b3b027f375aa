#!/usr/bin/env python3
"""What the per-signature A/R table traffic costs k_verify_dsm (GPU box).

Run once per library: the default build and the FD_DSM_TRAFFIC_PROBE
diagnostic builds (python firedancer_amd/build.py probe1
FD_DSM_TRAFFIC_PROBE=1; probe2 ... =2), selected with FD_ED25519_HIP_LIB.
The probes execute the same instructions but read (1) or also build (2) 64
shared, L2-resident tables, so their verdicts are wrong and only their
timing means anything.  On one C2 batch of 2^20 signatures (one context):
- dsm_ms / prep_ms: HIP-event launch times (timing mode), `reps` launches;
- sustained_ms: wall time per whole verify call over `secs` seconds of
  back-to-back calls, the power-capped steady state the bench runs in.

usage: python tools/dsm_traffic_probe.py [secs] [reps]   -> one JSON line
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    import torch
    from firedancer_amd import Verifier
    from firedancer_amd.ed25519 import CTX_STREAM
    from firedancer_amd.workload import make_batch_gpu
    n = 1 << 20
    v = Verifier(device=0, chunk_sigs=n)
    b = make_batch_gpu(v, n, msg_sz=64, seed=0x5eed0001, mix="c2")
    torch.cuda.synchronize()
    codes = torch.zeros(n, dtype=torch.int8, device=b.dev)

    def call():
        v.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes, stream=CTX_STREAM)

    for _ in range(3):
        call()
    v.sync()
    v.set_timing(True)
    for _ in range(reps):
        call()
    v.sync()
    prep_ms, dsm_ms, launches = v.get_timing()
    v.set_timing(False)
    k, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < secs:
        for _ in range(20):
            call()
        v.sync()
        k += 20
        print(f"{k} calls {time.perf_counter() - t0:.1f} s", file=sys.stderr)
    dt = time.perf_counter() - t0
    lib = os.path.basename(os.environ.get("FD_ED25519_HIP_LIB", "libfd_ed25519_hip.so"))
    print(json.dumps({"lib": lib, "dsm_ms": round(dsm_ms / launches, 3), "prep_ms": round(prep_ms / launches, 3),
                      "sustained_ms": round(dt / k * 1e3, 3), "calls": k,
                      "accept_rate": round(float((codes == 0).float().mean()), 4)}))
    v.close()


if __name__ == "__main__":
    main()
