#!/usr/bin/env python3
"""Latency-path launch time against the number of racing copies (product
build): n signatures per launch, set_lat_cus(cus) -> min(cus/n, 8) copies,
HIP events around each launch on the launch stream.  Prints p10/p50/p90 in
microseconds per (n, cus).  usage: python tools/lat_copies.py [reps]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    ns = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 12]
    cps = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 2, 4, 8]
    import torch
    from firedancer_amd import Verifier
    from firedancer_amd.workload import make_batch_gpu
    v = Verifier(device=0, chunk_sigs=4096)
    v.set_small_batch(256)
    out = {}
    for n in ns:
        b = make_batch_gpu(v, n, msg_sz=64, seed=11, mix="c1")
        codes = torch.empty(n, dtype=torch.int8, device="cuda")
        for cus in [max(c * n, 1) for c in cps]:
            v.set_lat_cus(cus)
            ts = []
            for r in range(reps + 3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                v.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes)
                e1.record()
                torch.cuda.synchronize()
                assert int((codes != 0).sum()) == 0
                if r >= 3:
                    ts.append(e0.elapsed_time(e1) * 1e3)
            p = np.percentile(ts, [10, 50, 90]).round(1).tolist()
            out[f"n{n}_copies{min(cus // n, 8)}"] = p
            print(f"n {n:3d} copies {min(cus // n, 8)}: us p10/50/90 {p}", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
