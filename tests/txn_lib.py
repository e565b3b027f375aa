"""ctypes bindings to the verify-tile oracle (oracle/liboracle.so: the plain-C
restatement) and to the reference's own verify-tile path built from its
sources (oracle/_ref/libfdref_txn.so) -- test infrastructure only.
"""
import ctypes
import os

import numpy as np

from oracle_lib import ERRMODE_AVX512, ORACLE_DIR, lib as oracle_lib

REF_TXN = os.path.join(ORACLE_DIR, "_ref", "libfdref_txn.so")
TXN_MAX_SZ = 852

c = ctypes
vp, u64, sz_t = c.c_void_p, c.c_uint64, c.c_size_t
_o = None
_r = None


class _TileState(c.Structure):
    _fields_ = [("hashmap_seed", u64), ("tcache_oldest", u64), ("tcache_ring", vp), ("tcache_depth", sz_t),
                ("tcache_map", vp), ("tcache_map_cnt", sz_t), ("bundle_failed", c.c_int), ("bundle_id", u64),
                ("parse_fail_cnt", u64), ("verify_fail_cnt", u64), ("dedup_fail_cnt", u64),
                ("bundle_peer_fail_cnt", u64)]


def olib():
    global _o
    if _o is None:
        L = oracle_lib()
        L.oracle_fd_hash.restype = u64
        L.oracle_fd_hash.argtypes = [u64, c.c_char_p, sz_t]
        L.oracle_txn_parse.restype = sz_t
        L.oracle_txn_parse.argtypes = [c.c_char_p, sz_t, vp]
        L.oracle_txn_parse_many.argtypes = [sz_t, vp, vp, vp, vp, vp]
        L.oracle_tcache_map_cnt_default.restype = sz_t
        L.oracle_tcache_map_cnt_default.argtypes = [sz_t]
        L.oracle_tcache_reset.argtypes = [vp, sz_t, vp, sz_t]
        L.oracle_tcache_query.restype = c.c_int
        L.oracle_tcache_query.argtypes = [vp, sz_t, u64]
        L.oracle_tcache_insert.restype = c.c_int
        L.oracle_tcache_insert.argtypes = [vp, vp, sz_t, vp, sz_t, u64]
        L.oracle_verify_tile_run.argtypes = [c.POINTER(_TileState), sz_t, vp, vp, vp, vp, vp, vp, vp, c.c_int]
        _o = L
    return _o


def have_ref():
    return os.path.exists(REF_TXN)


def rlib():
    global _r
    if _r is None:
        L = c.CDLL(REF_TXN)
        L.fd_hash.restype = u64
        L.fd_hash.argtypes = [u64, c.c_char_p, c.c_ulong]
        L.fd_txn_parse_core.restype = c.c_ulong
        L.fd_txn_parse_core.argtypes = [c.c_char_p, c.c_ulong, vp, vp, vp, c.c_ulong]
        L.ref_verify_tile_run.argtypes = [u64, vp, u64, vp, u64, vp, u64, vp, vp, vp, vp, vp, vp, vp, vp]
        L.ref_verify_tile_bench.argtypes = [c.c_int, c.c_int, u64, u64, u64, u64, vp, vp, vp, vp, vp]
        _r = L
    return _r


# ---- parse -------------------------------------------------------------------

def oracle_parse(payload):
    out = np.zeros(TXN_MAX_SZ, np.uint8)
    n = olib().oracle_txn_parse(bytes(payload), len(payload), out.ctypes.data)
    return n, out[:n].tobytes()


def ref_parse(payload):
    out = np.zeros(TXN_MAX_SZ + 64, np.uint8)
    n = rlib().fd_txn_parse_core(bytes(payload), len(payload), out.ctypes.data, None, None, 64)
    return n, out[:n].tobytes()


def oracle_parse_many(pool, off, sz, want_out=True):
    n = off.shape[0]
    pool = np.ascontiguousarray(pool, np.uint8)
    off = np.ascontiguousarray(off, np.uint32); sz = np.ascontiguousarray(sz, np.uint16)
    out = np.zeros((n, TXN_MAX_SZ), np.uint8) if want_out else None
    tsz = np.zeros(n, np.uint16)
    olib().oracle_txn_parse_many(n, pool.ctypes.data, off.ctypes.data, sz.ctypes.data,
                                 out.ctypes.data if want_out else None, tsz.ctypes.data)
    return tsz, out


# ---- verify tile ----------------------------------------------------------------

class OracleTile:
    def __init__(self, seed, depth, map_cnt=0, errmode=ERRMODE_AVX512):
        L = olib()
        self.depth = depth
        self.map_cnt = map_cnt or L.oracle_tcache_map_cnt_default(depth)
        self.ring = np.zeros(depth, np.uint64)
        self.map = np.zeros(self.map_cnt, np.uint64)
        self.st = _TileState(hashmap_seed=seed & (2**64 - 1), tcache_oldest=0, tcache_ring=self.ring.ctypes.data,
                             tcache_depth=depth, tcache_map=self.map.ctypes.data, tcache_map_cnt=self.map_cnt)
        self.errmode = errmode

    def reset_tcache(self):
        olib().oracle_tcache_reset(self.ring.ctypes.data, self.depth, self.map.ctypes.data, self.map_cnt)
        self.st.tcache_oldest = 0

    def run(self, pool, off, sz, bundle_id=None):
        n = off.shape[0]
        pool = np.ascontiguousarray(pool, np.uint8)
        off = np.ascontiguousarray(off, np.uint32); sz = np.ascontiguousarray(sz, np.uint16)
        bid = None if bundle_id is None else np.ascontiguousarray(bundle_id, np.uint64)
        res = np.zeros(n, np.int8); tag = np.zeros(n, np.uint64); tsz = np.zeros(n, np.uint16)
        olib().oracle_verify_tile_run(c.byref(self.st), n, pool.ctypes.data, off.ctypes.data, sz.ctypes.data,
                                      None if bid is None else bid.ctypes.data, res.ctypes.data, tag.ctypes.data,
                                      tsz.ctypes.data, self.errmode)
        return res, tag, tsz

    def metrics(self):
        s = self.st
        return dict(parse_fail_cnt=s.parse_fail_cnt, verify_fail_cnt=s.verify_fail_cnt,
                    dedup_fail_cnt=s.dedup_fail_cnt, bundle_peer_fail_cnt=s.bundle_peer_fail_cnt)

    @property
    def oldest(self):
        return int(self.st.tcache_oldest)


class RefTile:
    """The reference's fd_txn_verify + FD_TCACHE macros (header-inline, compiled
    from /root/reference) with after_frag's bookkeeping (ref_txn_drv.c)."""

    def __init__(self, seed, depth, map_cnt=0):
        self.seed = seed & (2**64 - 1)
        self.depth = depth
        self.map_cnt = map_cnt or olib().oracle_tcache_map_cnt_default(depth)
        self.ring = np.zeros(depth, np.uint64)
        self.map = np.zeros(self.map_cnt, np.uint64)
        self.state = np.zeros(3, np.uint64)        # oldest, bundle_failed, bundle_id
        self.m = np.zeros(4, np.uint64)

    def reset_tcache(self):
        self.ring[:] = 0; self.map[:] = 0; self.state[0] = 0

    def run(self, pool, off, sz, bundle_id=None):
        n = off.shape[0]
        pool = np.ascontiguousarray(pool, np.uint8)
        off = np.ascontiguousarray(off, np.uint32); sz = np.ascontiguousarray(sz, np.uint16)
        bid = None if bundle_id is None else np.ascontiguousarray(bundle_id, np.uint64)
        res = np.zeros(n, np.int8); tag = np.zeros(n, np.uint64); tsz = np.zeros(n, np.uint16)
        rlib().ref_verify_tile_run(self.seed, self.ring.ctypes.data, self.depth, self.map.ctypes.data, self.map_cnt,
                                   self.state.ctypes.data, n, pool.ctypes.data, off.ctypes.data, sz.ctypes.data,
                                   None if bid is None else bid.ctypes.data, res.ctypes.data, tag.ctypes.data,
                                   tsz.ctypes.data, self.m.ctypes.data)
        return res, tag, tsz

    def metrics(self):
        m = self.m
        return dict(parse_fail_cnt=int(m[0]), verify_fail_cnt=int(m[1]), dedup_fail_cnt=int(m[2]),
                    bundle_peer_fail_cnt=int(m[3]))

    @property
    def oldest(self):
        return int(self.state[0])


def oracle_signer(prvs, pool, msg_off, msg_sz):
    """signer() for make_txn_stream backed by the oracle (CPU tests)."""
    from oracle_lib import sign_many
    return sign_many(prvs, pool, msg_off, msg_sz)[:2]


def stream_frags(stream):
    return stream.pool, stream.off, stream.sz
