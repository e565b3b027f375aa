"""PCIe-inclusive rate of fd_ed25519_hip_verify_host (inputs and results in
host memory, pageable numpy arrays): C2 batch of 2^20 signatures with 64-B
messages, signed on the GPU and copied to the host first.  One JSON line.
Usage: python tools/bench_host.py [--steps K]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from firedancer_amd import Verifier  # noqa: E402
from firedancer_amd.workload import make_batch_gpu  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--n", type=int, default=1 << 20)
args = ap.parse_args()
n = args.n
v = Verifier(device=0, chunk_sigs=min(n, 1 << 20))
b = make_batch_gpu(v, n, msg_sz=64, seed=0x5eed0001, mix="c2")
sigs = b.sigs.cpu().numpy(); pubs = b.pubs.cpu().numpy(); pool = b.pool.cpu().numpy()
moff = b.msg_off.cpu().numpy().view(np.uint32); msz = b.msg_sz.cpu().numpy().view(np.uint32)
codes, bitmap = v.verify_host(sigs, pubs, pool, moff, msz)          # warm-up (staging allocation)
t0 = time.perf_counter()
for _ in range(args.steps):
    codes, bitmap = v.verify_host(sigs, pubs, pool, moff, msz)
dt = (time.perf_counter() - t0) / args.steps
in_bytes = sigs.nbytes + pubs.nbytes + pool.nbytes + moff.nbytes + msz.nbytes
print(json.dumps({"metric": "verify_host verifies/s (PCIe-inclusive, pageable host buffers)", "value": round(n / dt, 1),
                  "ms_per_batch": round(dt * 1e3, 3), "n": n, "h2d_bytes": int(in_bytes),
                  "d2h_bytes": int(codes.nbytes + bitmap.nbytes), "accept_rate": round(float((codes == 0).mean()), 5)}))
v.close()
