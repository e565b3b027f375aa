#!/usr/bin/env python3
"""Where does a lone k_verify_lat workgroup spend its time, per XCD?

Needs the diagnostic build (bash tools/build_lat_trace.sh: the product
sources with tools/lat_trace.patch, loaded through FD_ED25519_HIP_LIB;
FD_LAT_TRACE_RAW=<file> also dumps every workgroup's record): every copy of a
signature runs to completion and records s_memrealtime (100 MHz) at each
phase boundary.  Launches n signatures x 8 copies (one per XCD) `reps` times
and prints, per XCD, the median phase durations in microseconds:
  p1_w0/p1_w1/p1_w2  phase 1 per wave (decode A, decode R, hash + split)
  tab_w0/tab_w1      phase 2 table builds (A, R)
  p2_w0/p2_w1/p2_w2  phase 2 per wave (A chain, R chain, B chain) from the barrier
  total              first timestamp to the end of phase 3
  ghz                s_memtime ticks / realtime (core clock)
usage: FD_ED25519_HIP_LIB=... python tools/lat_trace.py [n] [reps]"""
import collections
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    import torch
    from firedancer_amd import Verifier
    from firedancer_amd.ed25519 import lib
    from firedancer_amd.workload import make_batch_gpu
    L = lib()
    L.fd_ed25519_hip_lat_trace.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
    v = Verifier(device=0, chunk_sigs=4096)
    v.set_small_batch(256)
    b = make_batch_gpu(v, n, msg_sz=64, seed=7, mix="c1")
    codes = torch.empty(n, dtype=torch.int8, device="cuda")
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    raw = []
    buf = np.zeros(n * 8 * 24, np.uint64)
    for r in range(reps + 2):
        v.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes)
        torch.cuda.synchronize()
        assert int((codes != 0).sum()) == 0
        assert L.fd_ed25519_hip_lat_trace(buf.ctypes.data, buf.size) == 0
        if r < 2:
            continue
        t = buf.reshape(-1, 24).astype(np.int64)
        for w in range(n * 8):
            x = t[w]
            t0 = x[2:5].min()
            us = lambda a, b0: (a - b0) / 100.0
            d = {"p1_w0": us(x[5], x[2]), "p1_w1": us(x[6], x[3]), "p1_w2": us(x[7], x[4]),
                 "tab_w0": us(x[8], x[5:8].max()), "tab_w1": us(x[9], x[5:8].max()),
                 "p2_w0": us(x[10], x[5:8].max()), "p2_w1": us(x[11], x[5:8].max()), "p2_w2": us(x[12], x[5:8].max()),
                 "total": us(x[13], t0), "ghz": (x[15] - x[14]) / max(x[13] - t0, 1) / 10.0}
            xcc = int(x[0])
            raw.append({"xcc": xcc, "hw": [int(x[16 + k]) for k in range(3)], "hw0": int(x[1]), **{k: round(float(val), 1) for k, val in d.items()}})
            for k, val in d.items():
                per[xcc][k].append(val)
            per[xcc]["cu"].append(int((x[1] >> 8) & 0xF) + 16 * int((x[1] >> 13) & 0x3))
            simds = [int((x[16 + k] >> 4) & 3) for k in range(3)]
            per[xcc]["distinct_simds"].append(len(set(simds)))
            simd_key = "same" if len(set(simds)) < 3 else "split"
            per[simd_key]["total"].append(d["total"]); per[simd_key]["p2_w0"].append(d["p2_w0"])
    raw_path = os.environ.get("FD_LAT_TRACE_RAW")
    if raw_path:
        with open(raw_path, "w") as f:
            json.dump(raw, f)
    out = {}
    for key in ("same", "split"):
        if key in per:
            print(f"working waves on {key} SIMDs: n {len(per[key]['total'])}, total p50 "
                  f"{np.median(per[key]['total']):.1f} us, A chain p50 {np.median(per[key]['p2_w0']):.1f} us")
    per.pop("same", None); per.pop("split", None)
    for xcc in sorted(per):
        out[xcc] = {k: round(float(np.median(vals)), 1) for k, vals in per[xcc].items() if k != "cu"}
        out[xcc]["p90_total"] = round(float(np.percentile(per[xcc]["total"], 90)), 1)
        out[xcc]["cus_seen"] = len(set(per[xcc]["cu"]))
        print(f"xcc {xcc}: " + " ".join(f"{k} {val}" for k, val in out[xcc].items()))
    print(json.dumps({"n": n, "reps": reps, "per_xcc": out}))


if __name__ == "__main__":
    main()
