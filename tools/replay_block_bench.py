#!/usr/bin/env python3
"""Block-path sigverify throughput: fd_executor_txn_verify
for a whole block at once on the engine, against the per-transaction drop-in
(16 concurrent 12-signature callers) and the reference's
CPU verify on the box's host cores (bench.py cpu_baseline).

For blocks of --txns transactions (C4 shapes: 1-12 signers, legacy, C2
mutation model, GPU-signed), one JSON line each:
  resident   fd_replay_hip_txn_verify_dev, payloads and descriptors in HBM
  host       fd_replay_hip_txn_verify_host from pinned host buffers (the
             patched replay tile's call: H2D copy, verify, D2H results)
  sched      (--sched) the whole block through the reference's scheduler
             with integration/fd_replay_hip.patch (integration/sched_run.c,
             hip mode): FEC ingest, parse, claims, packing, GPU batches,
             retirement -- one host thread, as the replay tile; skip_seconds
             is the same loop with claimed txns passed unverified (the
             scheduler's own cost), so seconds - skip_seconds is what GPU
             sigverify adds to the replay thread; bulk_s is the replay
             thread's time inside the sigverify step itself (claims,
             packing, launch, polls, retirement) and
             sigverify_stage_sig_per_s = sigs / bulk_s; medians of 5 runs
sig/s = signatures in the block / seconds (median over --reps).
usage: python tools/replay_block_bench.py [--txns 16384,98039] [--reps 20] [--sched]"""
import argparse
import json
import os
import statistics
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", default="16384,98039")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--sched", action="store_true")
    args = ap.parse_args()
    import torch
    from firedancer_amd import Verifier
    from firedancer_amd.replay import DESC_DTYPE, ReplayVerifier
    from firedancer_amd.txn_workload import gpu_signer, make_txn_stream
    v = Verifier(device=0, chunk_sigs=1 << 20)
    for n in (int(x) for x in args.txns.split(",")):
        s = make_txn_stream(n, gpu_signer(v), seed=0x7e70 + n, dup_frac=0.0, graft_frac=0.0, bad_frac=0.0, v0_frac=0.0)
        # descriptors from the generator's layout (legacy: sig at 1, message after the signatures)
        nsig = s.pool[s.off.astype(np.int64)]
        desc = np.zeros(n, DESC_DTYPE)
        desc["payload_off"], desc["payload_sz"] = s.off, s.sz
        desc["signature_off"], desc["signature_cnt"] = 1, nsig
        desc["message_off"] = 1 + 64 * nsig.astype(np.uint16)
        desc["acct_addr_off"] = desc["message_off"] + 4
        sigs = int(nsig.astype(np.int64).sum())
        rv = ReplayVerifier(v, n)
        d_pool = torch.from_numpy(np.concatenate([s.pool, np.zeros(16, np.uint8)])).to("cuda:0")
        d_desc = torch.from_numpy(desc.view(np.uint8)).to("cuda:0")
        d_res = torch.zeros(n, dtype=torch.int32, device="cuda:0")
        h_pool = torch.from_numpy(np.ascontiguousarray(s.pool)).pin_memory().numpy()
        h_desc = torch.from_numpy(desc.view(np.uint8)).pin_memory().numpy().view(DESC_DTYPE)
        h_res = torch.zeros(n, dtype=torch.int32).pin_memory().numpy()
        out = {"metric": "block sigverify (fd_executor_txn_verify per txn, whole block per call)", "txns": n,
               "sigs": sigs, "reps": args.reps}
        for leg in ("resident", "host"):
            ts = []
            for r in range(args.reps + 2):
                torch.cuda.synchronize()
                t = time.perf_counter()
                if leg == "resident":
                    rv.txn_verify_dev(n, d_pool, d_desc, d_res)
                    v.sync()
                else:
                    rv.txn_verify_host(n, h_pool, h_desc, h_res)
                    rv.wait()
                if r >= 2:
                    ts.append(time.perf_counter() - t)
            med = statistics.median(ts)
            out[leg] = {"ms": med * 1e3, "sig_per_s": sigs / med, "txn_per_s": n / med}
        assert np.array_equal(h_res, d_res.cpu().numpy())
        out["fail_frac"] = float((h_res != 0).mean())
        rv.close()
        if args.sched:
            from replay_io import block_fecs, block_stream, run_sched, write_block
            with tempfile.TemporaryDirectory() as td:
                pool2, off2, sz2, sigs2 = block_stream(n, gpu_signer(v), 0x7e70 + n, "none")
                bp = os.path.join(td, "block.bin")
                write_block(bp, block_fecs(pool2, off2, sz2))
                reps = 5
                res = run_sched("sched_run_hip", [dict(block=bp, mode=m, exec_cnt=8) for m in ("skip", "hip") * reps], td)
                skips = [r for r, _ in res[0::2]]
                hips = [r for r, _ in res[1::2]]

                def mid(rs, k):
                    return statistics.median(r[k] for r in rs)
                info = sorted(hips, key=lambda r: r["seconds"])[reps // 2]
                bulk_s = mid(hips, "bulk_s")
                out["sched"] = {"txns": len(off2), "sigs": sigs2, "reps": reps, "seconds": mid(hips, "seconds"),
                                "sig_per_s": sigs2 / mid(hips, "seconds"), "skip_seconds": mid(skips, "seconds"),
                                "scheduler_floor_sig_per_s": sigs2 / mid(skips, "seconds"),
                                "ingest_s": mid(hips, "ingest_s"), "skip_ingest_s": mid(skips, "ingest_s"),
                                "sigverify_done_s": mid(hips, "sigverify_done_s"),
                                "bulk_s": bulk_s, "sigverify_stage_sig_per_s": sigs2 / bulk_s,
                                "bulk_batches": info["bulk_batches"], "bulk_max": info["bulk_max"],
                                "sigs_bulk": info["sigs_bulk"], "sigs_exec": info["sigs_exec"],
                                "block_ended": info["block_ended"]}
        print(json.dumps(out), flush=True)
    v.close()


if __name__ == "__main__":
    main()
