"""Service-mode verify stage runs (integration/svc_tile_run.c with the GPU tile
integration/svc_run.c, or its CPU stand-in oracle/_ref/svc_mock) -- test
infrastructure.  The payload digest a consumer computes over the frags a
tile publishes, in order, is an fd_hash chain (util/fd_hash.c: XXH64):
digest = fd_hash( digest, payload, payload_sz ), starting at DIGEST0;
reference_digest computes it from the reference tile's output
(oracle/tile_drv.c's FDO1)."""
import os
import struct
import sys

import numpy as np
import xxhash

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
BUILD = os.path.join(REPO, "integration", "_build")
MOCK = os.path.join(REPO, "oracle", "_ref", "svc_mock")
DIGEST0 = 0x5eedd16e57


def digest_of(payloads):
    d = DIGEST0
    for p in payloads:
        d = xxhash.xxh64(p, seed=d).intdigest()
    return d


def reference_digest(fdo1):
    """digest and counts of a reference tile run (tile_io.read_fdo1 output)"""
    pays = []
    for _sig, _tsorig, b in fdo1["frags"]:
        psz, = struct.unpack_from("<H", b, 8)
        pays.append(b[80:80 + psz])
    m = fdo1["metrics"]
    return dict(digest=digest_of(pays), published=len(pays), parse_fail=int(m[0]), verify_fail=int(m[1]),
                dedup=int(m[2]), bundle_peer_fail=int(m[3]))


def tile_counts(t):
    """a tile's entry of a run's JSON line, in reference_digest's form"""
    return dict(digest=int(t["digest"], 16), published=t["published"], parse_fail=t["parse_fail"],
                verify_fail=t["verify_fail"], dedup=t["dedup"], bundle_peer_fail=t["bundle_peer_fail"])


def share_stream(path, s, bid, t, tiles, seed, depth):
    """the frags of tile t's round robin share (one link: seq = frag index)
    as a stream of their own, for the reference tile"""
    from tile_io import write_fdt1
    idx = np.arange(t, s.n, tiles)
    write_fdt1(path, s.pool, s.off[idx], s.sz[idx], bid[idx], seed, depth)


def run(stream, tiles, in_depth, logdir, env=None, svc_env=None, mock=False, timeout=240):
    import svc_bench as SB
    assert os.path.exists(SB.EXE), "integration/_build/svc_tile_run missing: run build() with /root/reference"
    env = dict(env or {}, SVC_RUN_DIGEST="1")                 # the consumers read and digest every frag
    return SB.run_one(stream, tiles, in_depth, timeout, logdir, env=env, svc_env=svc_env,
                      svc_exe=MOCK if mock else None)


def ref_share_digests(pool, off, sz, bid, tiles, seed, depth, threads=8, seed_step=1):
    """each tile's published sequence (digest, counts) from the reference's
    own parse and AVX-512 verify (oracle/_ref/libfdref_txn.so
    ref_verify_tile_digest): tile t's share of one link, tile seed
    seed + t*seed_step (svc_tile_run.c seeds tile t with the stream's seed + t)"""
    import ctypes as c
    L = c.CDLL(os.path.join(REPO, "oracle", "_ref", "libfdref_txn.so"))
    u64, vp = c.c_uint64, c.c_void_p
    L.ref_verify_tile_digest.argtypes = [u64, u64, u64, u64, u64, vp, vp, vp, vp, c.c_int, vp]
    pool = np.ascontiguousarray(pool, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    sz = np.ascontiguousarray(sz, np.uint16)
    bid = np.ascontiguousarray(bid, np.uint64) if bid is not None else None
    res = []
    for t in range(tiles):
        out = np.zeros(8, np.uint64)
        L.ref_verify_tile_digest(tiles, t, seed + t * seed_step, depth, len(off), pool.ctypes.data, off.ctypes.data,
                                 sz.ctypes.data, bid.ctypes.data if bid is not None else None, threads, out.ctypes.data)
        res.append(dict(digest=int(out[0]), published=int(out[1]), parse_fail=int(out[2]), verify_fail=int(out[3]),
                        dedup=int(out[4]), bundle_peer_fail=int(out[5]), sigs=int(out[6])))
    return res
