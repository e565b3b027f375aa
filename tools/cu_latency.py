#!/usr/bin/env python3
"""Lone latency-kernel workgroup time on each CU: the context's stream is
restricted to one CU (fd_ed25519_hip_ctx_set_cu_mask), one signature, one
copy, `reps` launches timed with HIP events.  Prints per CU index the median
and the share of launches under 400 us, and a JSON summary.
usage: python tools/cu_latency.py [reps] [cus]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    import torch
    from firedancer_amd import Verifier
    from firedancer_amd.ed25519 import CTX_STREAM
    from firedancer_amd.workload import make_batch_gpu
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    cus = range(int(sys.argv[2])) if len(sys.argv) > 2 else range(ncu)
    v = Verifier(device=0, chunk_sigs=4096)
    v.set_small_batch(256)
    v.set_lat_cus(1)                      # one copy
    b = make_batch_gpu(v, 1, msg_sz=64, seed=3, mix="c1")
    torch.cuda.synchronize()
    codes = torch.empty(1, dtype=torch.int8, device="cuda")
    out = {}
    for cu in cus:
        assert v.set_cu_mask([cu]) == 0
        s = torch.cuda.ExternalStream(v.stream, device="cuda")
        ts = []
        for r in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            v.verify_dev(1, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes, stream=CTX_STREAM)
            e1.record(s)
            e1.synchronize()
            assert int(codes[0]) == 0
            if r:
                ts.append(e0.elapsed_time(e1) * 1e3)
        out[cu] = {"p50_us": round(float(np.median(ts)), 1), "fast_share": round(float(np.mean(np.array(ts) < 400)), 2)}
        print(f"cu {cu:3d}: p50 {out[cu]['p50_us']:7.1f} us, fast {out[cu]['fast_share']:.2f}", flush=True)
    v.set_cu_mask(None)
    fast = [c for c, d in out.items() if d["fast_share"] >= 0.99]
    print(json.dumps({"reps": reps, "per_cu": out, "always_fast": fast}))


if __name__ == "__main__":
    main()
