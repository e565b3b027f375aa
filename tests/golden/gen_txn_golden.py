#!/usr/bin/env python3
"""Generate the verify-tile golden fixtures (tests/golden/txn_vectors.json,
tests/golden/c4_stream_2048.npz).

Runs ONLY in the build container: it reads data out of /root/reference and
loads the reference's own verify-tile path compiled by oracle/Makefile
(oracle/_ref/libfdref_txn.so: fd_txn_parse_core, fd_hash, fd_txn_verify with
the FD_TCACHE macros).  The fixtures are data: inputs and the reference's
outputs.  Nothing under -m gpu, smoke() or bench.py reads /root/reference.

Sources (paths relative to /root/reference):
  src/ballet/txn/fixtures/transaction{1..6}.bin   parse fixtures of test_txn_parse.c
  src/ballet/txn/test_txn_parse.c:250-259          their expected footprints
  src/disco/verify/test_verify.c:5-112              the txn hex strings
  src/disco/verify/test_verify.c:168-343            the fd_txn_verify call sequences
plus fd_hash vectors (random inputs, reference outputs) and a 2048-frag C4
stream (repo generator, oracle-signed) with the reference's per-frag results.

usage: python tests/golden/gen_txn_golden.py   (after `make -C oracle all`)
"""
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("FD_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)

import txn_lib as T  # noqa: E402
from firedancer_amd.txn_workload import make_txn_stream  # noqa: E402

# test_verify.c: the fd_txn_verify sequences as data.  Each step is
# (txn array name, dedup flag, expected FD_TXN_VERIFY_* code) or "reset"
# (fd_tcache_reset); each list runs on a fresh ctx (setup_verify_ctx: depth 16,
# map_cnt 64).
VERIFY_SEQS = {
    "test_verify_success": [                                    # :168-212
        ("valid_txn_2sigs", 1, 0), ("valid_txn_2sigs", 1, -2), ("valid_txn_2sigs", 1, -2),
        ("valid_txn_2sigs", 0, 0),
        ("valid_txn_1sig", 1, 0), ("valid_txn_1sig", 1, -2), ("valid_txn_1sig", 1, -2)],
    "test_verify_invalid_sigs_success": [                       # :214-240
        ("invalid_txn_2sigs", 1, -1), ("invalid_txn_2sigs", 1, -1)],
    "test_verify_invalid_dedup_success": [                      # :242-311
        ("invalid_txn_same_1sig", 1, -1), ("valid_txn_1sig", 1, 0), "reset",
        ("valid_txn_1sig", 1, 0), ("invalid_txn_same_1sig", 1, -2), "reset",
        ("valid_txn_1sig", 0, 0), ("invalid_txn_same_1sig", 0, -1), ("invalid_txn_same_1sig", 1, -1),
        ("invalid_txn_same_1sig", 1, -1)],
    "test_verify_invalid_dedup_with_collision_success": [       # :313-343
        ("valid_txn_1sig", 1, 0), ("invalid_txn_1sig_same_64bit", 1, -1)],
}


def verify_txns():
    src = open(os.path.join(REF, "src/disco/verify/test_verify.c")).read()
    out = {}
    for m in re.finditer(r"static char \*\s*(\w+)\[\]\s*=\s*\{(.*?)\};", src, re.S):
        parts = re.findall(r'"([0-9a-fA-F]*)"', m.group(2))
        out[m.group(1)] = "".join(parts).lower()
    return out


def run_seq_ref(txns, seq):
    """Replay a sequence on the reference build: dedup=1 -> plain frag, dedup=0
    -> a frag of its own one-txn bundle (after_frag passes dedup=!is_bundle)."""
    tile = T.RefTile(seed=0x1234, depth=16, map_cnt=64)
    got, bid = [], 1000
    for step in seq:
        if step == "reset":
            tile.reset_tcache(); continue
        name, dedup, _ = step
        p = np.frombuffer(bytes.fromhex(txns[name]), np.uint8)
        b = None if dedup else np.array([bid], np.uint64)
        bid += 1
        res, _, _ = tile.run(p, np.zeros(1, np.uint32), np.array([p.size], np.uint16), b)
        got.append(int(res[0]))
    return got


def main():
    assert T.have_ref(), "build oracle/_ref first: make -C oracle all"
    fx = {"parse": [], "verify_txns": {}, "verify_seqs": {}, "fd_hash": []}
    # parse fixtures
    expect = {3: 852, 4: 20, 5: 0, 6: 30}                     # test_txn_parse.c:250-259
    for k in range(1, 7):
        b = open(os.path.join(REF, f"src/ballet/txn/fixtures/transaction{k}.bin"), "rb").read()
        n, out = T.ref_parse(b)
        if k in expect:
            assert n == expect[k], (k, n)
        fx["parse"].append({"name": f"transaction{k}", "payload": b.hex(), "footprint": int(n), "txn_t": out.hex()})
    # verify sequences
    txns = verify_txns()
    fx["verify_txns"] = txns
    for name, seq in VERIFY_SEQS.items():
        got = run_seq_ref(txns, seq)
        want = [s[2] for s in seq if s != "reset"]
        assert got == want, (name, got, want)
        fx["verify_seqs"][name] = [s if s == "reset" else list(s) for s in seq]
    # fd_hash vectors
    rng = np.random.default_rng(0xfd4a5)
    for i in range(48):
        sz = 64 if i < 16 else int(rng.integers(0, 200))
        b = rng.integers(0, 256, sz, dtype=np.uint8).tobytes()
        seed = int(rng.integers(0, 2**63)) * 2 + (i & 1)
        fx["fd_hash"].append({"seed": str(seed), "in": b.hex(), "out": str(T.rlib().fd_hash(seed, b, sz))})
    with open(os.path.join(HERE, "txn_vectors.json"), "w") as f:
        json.dump(fx, f, indent=0)

    # C4 stream fixture: 2048 frags incl. bundles, reference per-frag results
    s = make_txn_stream(2048, T.oracle_signer, seed=0xc4f1, dup_frac=0.03, graft_frac=0.01, bad_frac=0.02)
    bid = np.zeros(s.n, np.uint64)
    r = np.random.default_rng(5)
    for start in r.choice(s.n - 8, 40, replace=False):
        bid[start:start + int(r.integers(1, 6))] = int(r.integers(1, 2**40))
    tile = T.RefTile(seed=0xdecafbad, depth=256, map_cnt=0)
    res, tag, tsz = tile.run(s.pool, s.off, s.sz, bid)
    np.savez_compressed(os.path.join(HERE, "c4_stream_2048.npz"), pool=s.pool, off=s.off, sz=s.sz, bundle_id=bid,
                        seed=np.uint64(0xdecafbad), depth=np.uint64(256), result=res, tag=tag, txn_t_sz=tsz,
                        metrics=np.array([tile.metrics()[k] for k in ("parse_fail_cnt", "verify_fail_cnt",
                                                                      "dedup_fail_cnt", "bundle_peer_fail_cnt")],
                                         np.uint64),
                        ring=tile.ring, map=tile.map, oldest=np.uint64(tile.oldest))
    print("results:", dict(zip(*[x.tolist() for x in np.unique(res, return_counts=True)])))


if __name__ == "__main__":
    main()
