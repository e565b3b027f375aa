#!/usr/bin/env python3
"""Per-phase timing of k_txnm_batch (diagnostic; GPU box).

Runs one C4 batch (bench.py's stream and frag layout) through one verify
tile on an FD_TXNM_TRACE build (python firedancer_amd/build.py txtr
FD_TXNM_TRACE=1; selected with FD_ED25519_HIP_LIB=txtr) and reads the
per-workgroup s_memtime stamps: T0 start, T1 metadata, T2 staged, T3 slow
path + copy/parse ordering, T4 parsed, T5 record range claimed + tag, T6
records written, T7 histogram.  Prints, per phase, the median and p90 of
the cycle counts, and the workgroups' lifetime against the launch span.

usage: FD_ED25519_HIP_LIB=txtr python tools/txnm_trace.py [frags]
       FD_TXNM_NO_TRACE=1 FD_ED25519_HIP_LIB=<variant> ...: kernel time only"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from firedancer_amd import Verifier
    from firedancer_amd.ed25519 import lib
    from firedancer_amd.txn_workload import PARSED_CHUNKS, gpu_signer, make_txn_stream, txnm_dcache
    from firedancer_amd.verify_tile import IN_QUIC, VerifyTile
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    fb = int(os.environ.get("FD_VERIFY_HIP_FB", "16"))
    v = Verifier(device=0, chunk_sigs=1 << 20)
    s = make_txn_stream(n, gpu_signer(v), seed=0x5eed0004)
    region, chunk, fsz = txnm_dcache(s.pool, s.off, s.sz, seed=1)
    dev = torch.device("cuda", 0)
    to = lambda a, view=None: torch.from_numpy(np.ascontiguousarray(a if view is None else a.view(view))).to(dev)
    d_in = to(region)
    d_out = torch.empty(64 * PARSED_CHUNKS * n, dtype=torch.uint8, device=dev)
    out_chunk = to((np.arange(n) * PARSED_CHUNKS).astype(np.uint32), np.int32)
    tile = VerifyTile(v, max_txn=n, hashmap_seed=7, tcache_depth=4194302)
    args = (n, d_in, to(chunk, np.int32), to(fsz, np.int16), to(np.full(n, IN_QUIC, np.uint8)), d_out, out_chunk)
    tile.set_ingest_timing(True)
    ms = []
    for k in range(4):
        tile.set_seed(7 + k)
        tile.submit_frags(*args)
        tile.complete()
        ms.append(tile.ingest_stats())
    st = ms[-1]
    kms = float(np.median([m["ms"] for m in ms[1:]]))
    if os.environ.get("FD_TXNM_NO_TRACE"):
        print(json.dumps({"frags": n, "kernel_ms": kms, "bytes": st["bytes"], "records": st["records"],
                          "GBps": st["bytes"] / kms / 1e6, "lib": os.environ.get("FD_ED25519_HIP_LIB")}))
        return
    L = lib()
    L.fd_verify_hip_txnm_trace.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
    wg = (n + fb - 1) // fb
    tr = np.zeros((wg, 8), np.uint64)
    assert L.fd_verify_hip_txnm_trace(tr.ctypes.data, wg) == 0
    tr = tr.astype(np.int64)
    d = np.diff(tr, axis=1)
    names = ["meta", "stage", "slowpath+order", "parse", "claim+tag", "records", "hist"]
    out = {"frags": n, "fb": fb, "workgroups": wg, "kernel_ms": kms, "bytes": st["bytes"],
           "GBps": st["bytes"] / kms / 1e6, "phases_cycles": {}}
    for i, nm in enumerate(names):
        out["phases_cycles"][nm] = {"p50": float(np.median(d[:, i])), "p90": float(np.percentile(d[:, i], 90)),
                                    "mean": float(d[:, i].mean())}
    life = tr[:, 7] - tr[:, 0]
    out["lifetime_cycles"] = {"p50": float(np.median(life)), "p90": float(np.percentile(life, 90))}
    # s_memtime counts per XCD; the launch span is taken per XCD (workgroups are dealt round robin)
    spans = []
    for x in range(8):
        t = tr[x::8]
        spans.append(int(t[:, 7].max() - t[:, 0].min()))
    out["span_cycles_per_xcd"] = spans
    out["wg_cycles_sum_over_span"] = float(life.sum() / 8 / np.median(spans))   # mean workgroups resident per XCD
    print(json.dumps(out))
    tile.close()
    v.close()


if __name__ == "__main__":
    main()
