"""Input/output files of oracle/tile_drv.c (the verify-tile driver) -- test
infrastructure.  FDT1: frags in; FDO1: published frags, metrics, tcache."""
import os
import struct
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = os.path.join(REPO, "oracle", "_ref")
TXNM_SZ = 80                      # sizeof(fd_txn_m_t), include/fd_verify_hip.h


def write_fdt1(path, pool, off, sz, bundle_id, seed, depth):
    n = len(off)
    with open(path, "wb") as f:
        f.write(b"FDT1")
        f.write(struct.pack("<QQQ", n, int(seed), int(depth)))
        for j in range(n):
            o, s = int(off[j]), int(sz[j])
            f.write(struct.pack("<QH", int(bundle_id[j]), s))
            f.write(np.asarray(pool[o:o + s], np.uint8).tobytes())


def read_fdo1(path, depth):
    b = open(path, "rb").read()
    assert b[:4] == b"FDO1"
    pub, = struct.unpack_from("<Q", b, 4)
    p, frags = 12, []
    for _ in range(pub):
        sig, sz, tsorig = struct.unpack_from("<QQQ", b, p)
        p += 24
        frags.append((sig, tsorig, b[p:p + sz]))
        p += sz
    met = np.frombuffer(b, np.uint64, 5, p).copy()
    p += 40
    oldest, = struct.unpack_from("<Q", b, p)
    p += 8
    ring = np.frombuffer(b, np.uint64, depth, p).copy()
    p += 8 * depth
    mp = np.frombuffer(b, np.uint64, (len(b) - p) // 8, p).copy()
    return dict(frags=frags, metrics=met, oldest=oldest, ring=ring, map=mp, raw=b)


def normalized(out):
    """The driver output with each frag's alignment pad (the byte between an
    odd-length payload and the 2-aligned fd_txn_t, fd_txn_m.h:101-104) left
    out: the reference tile never writes it, so it holds whatever an earlier
    frag left in the reused out chunk."""
    frags = []
    for sig, tsorig, b in out["frags"]:
        psz, = struct.unpack_from("<H", b, 8)
        at = (TXNM_SZ + psz + 1) & ~1
        frags.append((sig, tsorig, b[:TXNM_SZ + psz], b[at:]))
    return frags, out["metrics"].tobytes(), out["oldest"], out["ring"].tobytes(), out["map"].tobytes()


def run_driver(which, in_path, out_path, env=None, timeout=300):
    exe = os.path.join(REF_DIR, f"tile_drv_{which}")
    assert os.path.exists(exe), f"{exe} missing: run __graft_entry__.build() in the build container"
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run([exe, in_path, out_path], env=e, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    return r.stdout + r.stderr


def check_against_stream(out, pool, off, sz, result, txn_t_sz, metrics4):
    """The published frags are exactly the PUBLISH frags in arrival order,
    each the fd_txn_m_t header (payload_sz, txn_t_sz) + payload + fd_txn_t of
    its realized footprint; metrics as the reference's."""
    pub = np.array([t for _, t, _ in out["frags"]], np.int64)
    exp = np.nonzero(np.asarray(result) == 0)[0]
    assert np.array_equal(pub, exp), (pub.size, exp.size)
    for sig, t, b in out["frags"]:
        assert sig == 0
        psz, tsz = struct.unpack_from("<HH", b, 8)
        o, s = int(off[t]), int(sz[t])
        assert psz == s and tsz == int(txn_t_sz[t]), (t, psz, s, tsz, int(txn_t_sz[t]))
        assert b[TXNM_SZ:TXNM_SZ + s] == np.asarray(pool[o:o + s], np.uint8).tobytes(), t
        txn_at = (TXNM_SZ + s + 1) & ~1                  # fd_txn_m_txn_t: payload end, 2-aligned
        assert len(b) == txn_at + tsz, (t, len(b), txn_at, tsz)
    assert np.array_equal(out["metrics"][:4], np.asarray(metrics4, np.uint64)), (out["metrics"], metrics4)
