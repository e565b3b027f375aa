"""Block files for integration/sched_run.c (the reference's replay scheduler
with integration/fd_replay_hip.patch) and its output.

A block is the reference's entry-batch stream (fd_sched.c:1380-1420): each
batch is a u64 microblock count, then per microblock an fd_microblock_hdr_t
(src/ballet/block/fd_microblock.h:9-21: hash_cnt u64, hash[32], txn_cnt u64,
packed, 48 bytes) followed by txn_cnt serialized transactions.  A batch is
cut into FEC sets (fd_store_fec_t payloads) of at most fec_max bytes; a
batch's last FEC set carries is_last_in_batch."""
import os
import struct
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(os.path.dirname(HERE), "integration", "_build")
REC_DTYPE = np.dtype([("sig0", "u1", (64,)), ("result", "<i4"), ("source", "u1"), ("_pad", "u1", (3,))])
assert REC_DTYPE.itemsize == 72


def block_fecs(pool, off, sz, txn_per_mblk=48, mblk_per_batch=16, fec_max=31840, seed=5):
    """[(bytes, last_in_batch)] for the txns pool[off[i]:off[i]+sz[i]] in order."""
    rng = np.random.default_rng(seed)
    n, i, fecs = len(off), 0, []
    while i < n:
        parts, mb = [], 0
        while i < n and mb < mblk_per_batch:
            k = min(n - i, txn_per_mblk)
            parts.append(struct.pack("<Q", int(rng.integers(1, 12500))) + rng.bytes(32) + struct.pack("<Q", k))
            parts.extend(pool[int(off[j]):int(off[j]) + int(sz[j])].tobytes() for j in range(i, i + k))
            i, mb = i + k, mb + 1
        batch = struct.pack("<Q", mb) + b"".join(parts)
        cuts = list(range(0, len(batch), fec_max))
        for c in cuts:
            fecs.append((batch[c:c + fec_max], c == cuts[-1]))
    return fecs


def distinct_accounts(pool, off, sz):
    """Mask of the legacy txns whose account addresses are pairwise distinct.
    The C2 mutation model can give two signers of one txn the same
    small-order key; a txn that names an account twice never sanitizes on
    chain, and the reference's dispatcher (fd_rdisp) waits on itself for it,
    so such txns stay out of generated blocks."""
    keep = np.ones(len(off), bool)
    for i, (o, z) in enumerate(zip(off, sz)):
        p = pool[int(o):int(o) + int(z)]
        n = int(p[0])
        cnt = int(p[1 + 64 * n + 3])
        a = p[1 + 64 * n + 4:1 + 64 * n + 4 + 32 * cnt].reshape(cnt, 32)
        keep[i] = len(np.unique(a, axis=0)) == cnt
    return keep


def block_stream(n, signer, seed, mix, bad_at=None):
    """(pool, off, sz, signatures): n generated legacy txns (1-12 signers,
    mix "c2" or all valid) minus those naming an account twice, in block
    order; bad_at flips a bit of that txn's first signature."""
    from firedancer_amd.txn_workload import make_txn_stream
    s = make_txn_stream(n, signer, seed=seed, mix=mix, dup_frac=0.0, graft_frac=0.0, bad_frac=0.0, v0_frac=0.0)
    keep = distinct_accounts(s.pool, s.off, s.sz)
    off, sz, pool = s.off[keep], s.sz[keep], s.pool.copy()
    if bad_at is not None:
        pool[int(off[bad_at]) + 1 + 7] ^= 0x04
    return pool, off, sz, int(pool[off.astype(np.int64)].astype(np.int64).sum())


def write_block(path, fecs):
    with open(path, "wb") as f:
        f.write(b"FDB1" + struct.pack("<Q", len(fecs)))
        for data, last in fecs:
            f.write(struct.pack("<IB", len(data), int(last)) + data)


def read_records(path):
    with open(path, "rb") as f:
        assert f.read(4) == b"FDR1"
        (n,) = struct.unpack("<Q", f.read(8))
        return np.frombuffer(f.read(n * REC_DTYPE.itemsize), REC_DTYPE)


def run_sched(exe, jobs, tmp_dir, timeout=900):
    """Runs sched_run over jobs (dicts: block, mode, and optionally exec_cnt,
    record, batch_max, batch_min) in ONE process (the scheduler's memory is
    set up once); returns [(JSON summary, sigverify records)] in job order."""
    import json
    lines, outs = [], []
    for k, j in enumerate(jobs):
        out = os.path.join(str(tmp_dir), f"job{k}.bin")
        outs.append(out)
        lines.append(" ".join(str(x) for x in (j["block"], j["mode"], j.get("exec_cnt", 4), int(j.get("record", 0)), out,
                                               j.get("batch_max", 16384), j.get("batch_min", 256))))
    jf = os.path.join(str(tmp_dir), "jobs.txt")
    with open(jf, "w") as f:
        f.write("\n".join(lines) + "\n")
    r = subprocess.run([os.path.join(BUILD, exe), jf], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    infos = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(infos) == len(jobs), r.stdout[-2000:]
    return [(i, read_records(o)) for i, o in zip(infos, outs)]


def results_by_sig0(recs):
    """{sig0 bytes: result} (the blocks' sig0 are unique)."""
    d = {bytes(r["sig0"]): int(r["result"]) for r in recs}
    assert len(d) == len(recs), "duplicate sig0 in the records"
    return d


def sched_jobs_file(jobs, tmp_dir):
    """jobs.txt for sched_run (one job per line) and the records' paths"""
    lines, outs = [], []
    for k, j in enumerate(jobs):
        out = os.path.join(str(tmp_dir), f"job{k}.bin")
        outs.append(out)
        lines.append(" ".join(str(x) for x in (j["block"], j["mode"], j.get("exec_cnt", 4), int(j.get("record", 0)), out,
                                               j.get("batch_max", 16384), j.get("batch_min", 256))))
    jf = os.path.join(str(tmp_dir), "jobs.txt")
    with open(jf, "w") as f:
        f.write("\n".join(lines) + "\n")
    return jf, outs


def run_sched_svc(jobs, tmp_dir, mock=False, timeout=600, svc_env=None):
    """The svc-mode jobs (mode "svc") in ONE sched_run_svc process, a client
    of the GPU tile (integration/svc_run.c, or oracle/_ref/svc_mock with
    mock) in a clients-only run (svc_tile_run host, tools/svc_bench.py
    run_host).  Returns ([(JSON summary, records)] in job order, the host's
    line)."""
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(BUILD), "..", "tools"))
    import svc_bench as SB
    import svc_io as SI
    jf, outs = sched_jobs_file(jobs, tmp_dir)
    res = SB.run_host([("replay", [os.path.join(BUILD, "sched_run_svc"), jf])], os.path.join(str(tmp_dir), "logs"),
                      timeout=timeout, svc_exe=SI.MOCK if mock else None, svc_env=svc_env)
    infos = [json.loads(x) for x in res["clients_lines"]["replay"] if x.startswith("{")]
    assert len(infos) == len(jobs), res["clients_lines"]["replay"][-5:]
    return [(i, read_records(o)) for i, o in zip(infos, outs)], res
