"""Host-side mirror of the reference verify tile's per-frag path, backed by the
gfx950 engine (C ABI: include/fd_verify_hip.h, same library as ed25519.py).

Reference interface it mirrors:
  fd_txn_parse          src/ballet/txn/fd_txn.h:712-715 (fd_txn_parse.c:7-254)
  fd_hash               src/util/fd_hash.c:14-72
  fd_txn_verify         src/disco/verify/fd_verify_tile.h:61-111
                        (codes FD_TXN_VERIFY_SUCCESS / FAILED / DEDUP, :9-11)
  after_frag            src/disco/verify/fd_verify_tile.c:101-161
  tcache                src/tango/tcache/fd_tcache.h

`VerifyTile.after_frags` takes a batch of frags in arrival order and returns,
per frag, what after_frag would have done with it (publish, or which metric
it bumped), the dedup tag published with it and the fd_txn_t footprint.
There is no CPU fallback: everything runs through the HIP library.
"""
import ctypes

import numpy as np

from .ed25519 import Verifier, _ptr, lib as _ed_lib

FD_TXN_MAX_SZ = 852
FD_TXN_MTU = 1232
FD_TXN_VERIFY_SUCCESS, FD_TXN_VERIFY_FAILED, FD_TXN_VERIFY_DEDUP = 0, -1, -2

FRAG_PUBLISH = 0
FRAG_VERIFY_FAIL = -1
FRAG_DEDUP = -2
FRAG_PARSE_FAIL = -3
FRAG_BUNDLE_PEER = -4

# Every symbol include/fd_verify_hip.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "fd_txn_hip_parse_dev", "fd_verify_hip_hash", "fd_verify_hip_tcache_map_cnt_default",
    "fd_verify_hip_tcache_reset", "fd_verify_hip_tcache_query", "fd_verify_hip_tcache_insert",
    "fd_verify_hip_tile_new", "fd_verify_hip_tile_join_tcache", "fd_verify_hip_tile_tcache_reset",
    "fd_verify_hip_tile_delete", "fd_verify_hip_tile_set_seed", "fd_verify_hip_tile_submit", "fd_verify_hip_tile_complete",
    "fd_verify_hip_tile_complete_skip", "fd_verify_hip_tile_submit_range", "fd_verify_hip_tile_complete_range",
    "fd_verify_hip_tile_set_staging", "fd_verify_hip_tile_set_cu_mask",
    "fd_verify_hip_tile_metrics", "fd_verify_hip_tile_metrics2", "fd_verify_hip_tile_last_timing", "fd_verify_hip_tile_submit_frags",
    "fd_verify_hip_before_frag", "fd_verify_hip_hist_edges", "fd_verify_hip_tile_hist_init",
    "fd_verify_hip_tile_hist", "fd_verify_hip_tile_poll", "fd_verify_hip_tile_inflight",
    "fd_verify_hip_tile_set_ingest_timing", "fd_verify_hip_tile_ingest_stats", "fd_verify_hip_tile_set_inflight",
)
HIST_BUCKET_CNT = 16

# fd_txn_m_t / gossip vote layouts (include/fd_verify_hip.h)
TXNM_SZ, TXNM_PAYLOAD_SZ_OFF, TXNM_TXN_T_SZ_OFF, TXNM_SRC_IPV4_OFF, TXNM_SRC_TPU_OFF, TXNM_BUNDLE_ID_OFF = 80, 8, 10, 12, 16, 24
TPU_RAW_MTU, TPU_SOURCE_GOSSIP = 1312, 3
GOSSIP_UPDATE_TAG_VOTE, GOSSIP_VOTE_ADDR_OFF, GOSSIP_VOTE_TXN_SZ_OFF, GOSSIP_VOTE_TXN_OFF = 3, 56, 72, 80
IN_QUIC, IN_BUNDLE, IN_GOSSIP, IN_SEND = 0, 1, 2, 3
IN_HOSTCOPY = 0x80      # or'd into a kind: the host did during_frag's copy into the out chunk
FRAG_OVERRUN = -5       # complete_skip's result for a skipped (overrun) frag


class Range(ctypes.Structure):
    """fd_verify_hip_range_t: a published seq range of an unpolled in link's mcache."""
    _fields_ = [("mcache", ctypes.c_void_p), ("depth", ctypes.c_ulong), ("seq0", ctypes.c_ulong),
                ("seq_cnt", ctypes.c_ulong), ("rr_cnt", ctypes.c_ulong), ("rr_idx", ctypes.c_ulong),
                ("chunk_off", ctypes.c_ulong), ("chunk0", ctypes.c_ulong), ("wmark", ctypes.c_ulong)]


def range_frag_cnt(seq0, seq_cnt, rr_cnt, rr_idx):
    """fd_verify_hip_range_frag_cnt: seqs of [seq0, seq0+seq_cnt) with seq % rr_cnt == rr_idx."""
    if not seq_cnt or not rr_cnt or rr_idx >= rr_cnt:
        return 0
    first = seq0 + (rr_idx + rr_cnt - seq0 % rr_cnt) % rr_cnt
    end = seq0 + seq_cnt
    return (end - 1 - first) // rr_cnt + 1 if first < end else 0

_bound = False


def lib():
    global _bound
    L = _ed_lib()
    if not _bound:
        c = ctypes
        vp, u64 = c.c_void_p, c.c_ulong
        L.fd_txn_hip_parse_dev.restype = c.c_int
        L.fd_txn_hip_parse_dev.argtypes = [vp, u64, vp, vp, vp, vp, vp, vp]
        L.fd_verify_hip_hash.restype = u64
        L.fd_verify_hip_hash.argtypes = [u64, c.c_char_p, u64]
        L.fd_verify_hip_tcache_map_cnt_default.restype = u64
        L.fd_verify_hip_tcache_map_cnt_default.argtypes = [u64]
        L.fd_verify_hip_tcache_reset.restype = u64
        L.fd_verify_hip_tcache_reset.argtypes = [vp, u64, vp, u64]
        L.fd_verify_hip_tcache_query.restype = c.c_int
        L.fd_verify_hip_tcache_query.argtypes = [vp, u64, u64]
        L.fd_verify_hip_tcache_insert.restype = c.c_int
        L.fd_verify_hip_tcache_insert.argtypes = [vp, vp, u64, vp, u64, u64]
        L.fd_verify_hip_tile_new.restype = vp
        L.fd_verify_hip_tile_new.argtypes = [vp, u64, u64, u64, u64]
        L.fd_verify_hip_tile_join_tcache.argtypes = [vp, vp, vp, u64, vp, u64]
        L.fd_verify_hip_tile_tcache_reset.argtypes = [vp]
        L.fd_verify_hip_tile_delete.argtypes = [vp]
        L.fd_verify_hip_tile_set_seed.argtypes = [vp, u64]
        L.fd_verify_hip_tile_submit.restype = c.c_int
        L.fd_verify_hip_tile_submit.argtypes = [vp, u64, vp, vp, vp, vp]
        L.fd_verify_hip_tile_complete.restype = c.c_int
        L.fd_verify_hip_tile_poll.restype = c.c_int
        L.fd_verify_hip_tile_poll.argtypes = [vp]
        L.fd_verify_hip_tile_inflight.restype = u64
        L.fd_verify_hip_tile_inflight.argtypes = [vp]
        L.fd_verify_hip_tile_complete.argtypes = [vp, vp, vp, vp, vp]
        L.fd_verify_hip_tile_complete_skip.restype = c.c_int
        L.fd_verify_hip_tile_complete_skip.argtypes = [vp, vp, vp, vp, vp, vp]
        L.fd_verify_hip_tile_metrics.argtypes = [vp, vp]
        L.fd_verify_hip_tile_metrics2.argtypes = [vp, vp]
        L.fd_verify_hip_tile_last_timing.argtypes = [vp, vp]
        L.fd_verify_hip_tile_set_ingest_timing.argtypes = [vp, c.c_int]
        L.fd_verify_hip_tile_ingest_stats.argtypes = [vp, vp]
        L.fd_verify_hip_tile_set_inflight.restype = c.c_int
        L.fd_verify_hip_tile_set_inflight.argtypes = [vp, u64]
        L.fd_verify_hip_tile_submit_frags.restype = c.c_int
        L.fd_verify_hip_tile_submit_frags.argtypes = [vp, u64, vp, vp, vp, vp, vp, vp]
        L.fd_verify_hip_tile_submit_range.restype = c.c_int
        L.fd_verify_hip_tile_submit_range.argtypes = [vp, c.POINTER(Range), vp, vp, vp]
        L.fd_verify_hip_tile_complete_range.restype = c.c_int
        L.fd_verify_hip_tile_set_staging.restype = c.c_int
        L.fd_verify_hip_tile_set_staging.argtypes = [vp, c.c_int]
        L.fd_verify_hip_tile_set_cu_mask.restype = c.c_int
        L.fd_verify_hip_tile_set_cu_mask.argtypes = [vp, vp, c.c_uint]
        L.fd_verify_hip_tile_complete_range.argtypes = [vp, vp, vp, vp, vp, vp]
        L.fd_verify_hip_before_frag.restype = c.c_int
        L.fd_verify_hip_before_frag.argtypes = [c.c_uint, u64, u64, u64, u64]
        L.fd_verify_hip_hist_edges.restype = c.c_int
        L.fd_verify_hip_hist_edges.argtypes = [u64, u64, vp]
        L.fd_verify_hip_tile_hist_init.restype = c.c_int
        L.fd_verify_hip_tile_hist_init.argtypes = [vp, u64, u64]
        L.fd_verify_hip_tile_hist.restype = c.c_int
        L.fd_verify_hip_tile_hist.argtypes = [vp, c.c_int, vp, vp, vp]
        _bound = True
    return L


def fd_hash(seed, buf):
    """util/fd_hash.c:14-72 (host entry of the engine; the GPU computes the same)."""
    b = bytes(buf)
    return lib().fd_verify_hip_hash(int(seed) & (2**64 - 1), b, len(b))


class Tcache:
    """A tcache in the reference layout (ring[depth], map[map_cnt], oldest)."""

    def __init__(self, depth, map_cnt=0):
        L = lib()
        self.depth = int(depth)
        self.map_cnt = int(map_cnt) or int(L.fd_verify_hip_tcache_map_cnt_default(self.depth))
        self.ring = np.zeros(self.depth, np.uint64)
        self.map = np.zeros(self.map_cnt, np.uint64)
        self.oldest = np.zeros(1, np.uint64)
        self.reset()

    def reset(self):
        self.oldest[0] = lib().fd_verify_hip_tcache_reset(self.ring.ctypes.data, self.depth, self.map.ctypes.data,
                                                          self.map_cnt)

    def query(self, tag):
        return bool(lib().fd_verify_hip_tcache_query(self.map.ctypes.data, self.map_cnt, int(tag)))

    def insert(self, tag):
        return bool(lib().fd_verify_hip_tcache_insert(self.oldest.ctypes.data, self.ring.ctypes.data, self.depth,
                                                      self.map.ctypes.data, self.map_cnt, int(tag)))


def parse_dev(verifier, n, pool, txn_off, txn_sz, txn_out, txn_t_sz, stream=None):
    """fd_txn_parse over n device-resident payloads (torch tensors / pointers)."""
    n, dev = int(n), verifier.device
    args = (verifier.ctx, n, _ptr(pool, 1, "pool", dev), _ptr(txn_off, 4 * n, "txn_off", dev),
            _ptr(txn_sz, 2 * n, "txn_sz", dev), _ptr(txn_out, 0, "txn_out", dev), _ptr(txn_t_sz, 2 * n, "txn_t_sz", dev))
    with verifier._stream(stream) as h:
        return lib().fd_txn_hip_parse_dev(*args, h)


def hist_edges(min_v, max_v):
    """The 16 left edges fd_histf_new(min_v, max_v) gives (fd_histf.h:88-118);
    ValueError if max_v <= min_v."""
    edge = np.zeros(HIST_BUCKET_CNT, np.uint64)
    if lib().fd_verify_hip_hist_edges(int(min_v), int(max_v), edge.ctypes.data):
        raise ValueError("max_v must exceed min_v")
    return edge


def before_frag(in_kind, seq, sig, round_robin_cnt, round_robin_idx):
    """fd_verify_tile.c:37-58: True if this tile skips the frag."""
    return bool(lib().fd_verify_hip_before_frag(int(in_kind), int(seq), int(sig) & (2**64 - 1),
                                                int(round_robin_cnt), int(round_robin_idx)))


class VerifyTile:
    """One verify tile on one GPU: fd_verify_ctx_t's tcache, hashmap_seed,
    bundle state and metrics, with frags processed in device-resident batches."""

    def __init__(self, verifier=None, max_txn=1 << 16, hashmap_seed=0, tcache_depth=4194302, tcache_map_cnt=0,
                 device=0, chunk_sigs=1 << 20):
        self._lib = lib()
        self.verifier = verifier if verifier is not None else Verifier(device=device, chunk_sigs=chunk_sigs)
        self.max_txn = int(max_txn)
        self.tile = self._lib.fd_verify_hip_tile_new(self.verifier.ctx, self.max_txn, int(hashmap_seed) & (2**64 - 1),
                                                     int(tcache_depth), int(tcache_map_cnt))
        if not self.tile:
            raise RuntimeError("fd_verify_hip_tile_new failed (bad tcache depth / map_cnt?)")
        self._joined = None
        self._pending = []

    def join_tcache(self, tc: Tcache):
        """Use an external tcache (the reference tile's ctx->tcache_* arrays)."""
        self._joined = tc
        self._lib.fd_verify_hip_tile_join_tcache(self.tile, tc.oldest.ctypes.data, tc.ring.ctypes.data, tc.depth,
                                                 tc.map.ctypes.data, tc.map_cnt)

    def tcache_reset(self):
        self._lib.fd_verify_hip_tile_tcache_reset(self.tile)

    def set_seed(self, seed):
        self._lib.fd_verify_hip_tile_set_seed(self.tile, int(seed) & (2**64 - 1))

    def submit(self, n, pool, txn_off, txn_sz, txn_out=None):
        """Device tensors: pool uint8, txn_off int32 (u32 bits), txn_sz int16 (u16 bits)."""
        n, dev = int(n), self.verifier.device
        rc = self._lib.fd_verify_hip_tile_submit(self.tile, n, _ptr(pool, 1, "pool", dev),
                                                 _ptr(txn_off, 4 * n, "txn_off", dev),
                                                 _ptr(txn_sz, 2 * n, "txn_sz", dev), _ptr(txn_out, 0, "txn_out", dev))
        if rc:
            raise RuntimeError(f"fd_verify_hip_tile_submit: {rc}")
        self._pending.append((int(n), (pool, txn_off, txn_sz, txn_out)))   # keep buffers alive

    def submit_frags(self, n, d_in, in_chunk, in_sz, in_kind, d_out, out_chunk):
        """fd_txn_m_t frag batch (fd_verify_hip_tile_submit_frags): device tensors
        d_in / d_out uint8 dcache regions, in_chunk / out_chunk int32 (u32 64-B
        chunk indices), in_sz int16 (u16 frag sizes), in_kind uint8 (IN_*)."""
        n, dev = int(n), self.verifier.device
        rc = self._lib.fd_verify_hip_tile_submit_frags(
            self.tile, n, _ptr(d_in, 1, "d_in", dev), _ptr(in_chunk, 4 * n, "in_chunk", dev),
            _ptr(in_sz, 2 * n, "in_sz", dev), _ptr(in_kind, n, "in_kind", dev), _ptr(d_out, 1, "d_out", dev),
            _ptr(out_chunk, 4 * n, "out_chunk", dev))
        if rc:
            raise RuntimeError(f"fd_verify_hip_tile_submit_frags: {rc}")
        self._pending.append((n, (d_in, in_chunk, in_sz, in_kind, d_out, out_chunk)))

    def submit_range(self, mcache, depth, seq0, seq_cnt, rr_cnt, rr_idx, chunk_off, chunk0, wmark, d_in, d_out,
                     out_chunk):
        """fd_verify_hip_tile_submit_range: the GPU reads mcache lines [seq0, seq0+seq_cnt)
        (device tensor of depth 32-byte fd_frag_meta_t lines), keeps seq % rr_cnt == rr_idx
        and ingests those frags from d_in + 64*(chunk - chunk_off) into d_out + 64*out_chunk[j]."""
        dev = self.verifier.device
        n = range_frag_cnt(int(seq0), int(seq_cnt), int(rr_cnt), int(rr_idx))
        r = Range(_ptr(mcache, 32 * int(depth), "mcache", dev), int(depth), int(seq0), int(seq_cnt), int(rr_cnt),
                  int(rr_idx), int(chunk_off), int(chunk0), int(wmark))
        rc = self._lib.fd_verify_hip_tile_submit_range(self.tile, ctypes.byref(r), _ptr(d_in, 1, "d_in", dev),
                                                       _ptr(d_out, 1, "d_out", dev),
                                                       _ptr(out_chunk, 4 * max(n, 1), "out_chunk", dev))
        if rc:
            raise RuntimeError(f"fd_verify_hip_tile_submit_range: {rc}")
        self._pending.append((n, (mcache, d_in, d_out, out_chunk)))
        return n

    def complete_range(self, skip=None):
        """complete_skip plus each kept frag's mcache tsorig (range batches):
        (result, txn_t_sz, payload_sz, tsorig)."""
        n, _keep = self._pending.pop(0)
        sk = None if skip is None else np.ascontiguousarray(skip, np.uint8)
        assert sk is None or sk.size >= n
        result = np.zeros(max(n, 1), np.int8)
        tsz = np.zeros(max(n, 1), np.uint16)
        psz = np.zeros(max(n, 1), np.uint16)
        tso = np.zeros(max(n, 1), np.uint32)
        rc = self._lib.fd_verify_hip_tile_complete_range(self.tile, None if sk is None else sk.ctypes.data,
                                                         result.ctypes.data, tsz.ctypes.data, psz.ctypes.data,
                                                         tso.ctypes.data)
        if rc:
            raise RuntimeError(f"fd_verify_hip_tile_complete_range: {rc}")
        return result[:n], tsz[:n], psz[:n], tso[:n]

    def poll(self):
        """fd_verify_hip_tile_poll: 1 oldest batch done, 0 running, -1 none (never blocks)."""
        return int(self._lib.fd_verify_hip_tile_poll(self.tile))

    def inflight(self):
        return int(self._lib.fd_verify_hip_tile_inflight(self.tile))

    def complete(self, bundle_id=None):
        n, _keep = self._pending.pop(0)
        result = np.zeros(n, np.int8)
        tag = np.zeros(n, np.uint64)
        tsz = np.zeros(n, np.uint16)
        bid = None
        if bundle_id is not None:
            bid = np.ascontiguousarray(bundle_id, np.uint64)
            assert bid.shape == (n,)
        rc = self._lib.fd_verify_hip_tile_complete(self.tile, None if bid is None else bid.ctypes.data,
                                                   result.ctypes.data, tag.ctypes.data, tsz.ctypes.data)
        if rc:
            raise RuntimeError(f"fd_verify_hip_tile_complete: {rc}")
        return result, tag, tsz

    def complete_skip(self, skip):
        """complete() with skip[j] != 0 frags treated as overrun (FRAG_OVERRUN)."""
        n, _keep = self._pending.pop(0)
        skip = np.ascontiguousarray(skip, np.uint8)
        assert skip.size >= n
        result = np.zeros(n, np.int8)
        tag = np.zeros(n, np.uint64)
        tsz = np.zeros(n, np.uint16)
        psz = np.zeros(n, np.uint16)
        rc = self._lib.fd_verify_hip_tile_complete_skip(self.tile, skip.ctypes.data, result.ctypes.data,
                                                        tag.ctypes.data, tsz.ctypes.data, psz.ctypes.data)
        if rc:
            raise RuntimeError(f"fd_verify_hip_tile_complete_skip: {rc}")
        self.last_payload_sz = psz
        return result, tag, tsz

    def after_frags(self, n, pool, txn_off, txn_sz, bundle_id=None, txn_out=None):
        self.submit(n, pool, txn_off, txn_sz, txn_out)
        return self.complete(bundle_id)

    def metrics(self):
        out = np.zeros(7, np.uint64)
        self._lib.fd_verify_hip_tile_metrics2(self.tile, out.ctypes.data)
        keys = ("parse_fail_cnt", "verify_fail_cnt", "dedup_fail_cnt", "bundle_peer_fail_cnt", "published", "sigs",
                "gossiped_votes_cnt")
        return dict(zip(keys, (int(x) for x in out)))

    def last_timing(self):
        out = np.zeros(3, np.float64)
        self._lib.fd_verify_hip_tile_last_timing(self.tile, out.ctypes.data)
        return {"gpu_ms": float(out[0]), "host_ms": float(out[1]), "sigs": int(out[2])}

    def set_inflight(self, k):
        """Batches kept on the GPU at once (1..8; 2 for a new tile)."""
        if self._lib.fd_verify_hip_tile_set_inflight(self.tile, int(k)):
            raise ValueError("set_inflight: k out of range or batches outstanding")

    def set_staging(self, on=True):
        """Out staging (fd_verify_hip_tile_set_staging): batches work on HBM staging frags and
        write the out dcache at the end, only the bytes the reference writes."""
        if self._lib.fd_verify_hip_tile_set_staging(self.tile, int(bool(on))):
            raise ValueError("set_staging: batches outstanding or the split ingest")

    def set_ingest_timing(self, on=True):
        """HIP events around each batch's ingest kernel (k_txnm_batch)."""
        self._lib.fd_verify_hip_tile_set_ingest_timing(self.tile, int(bool(on)))

    def ingest_stats(self):
        """Last completed frag batch: ingest kernel ms (timing on), frags,
        algorithmic bytes (include/fd_verify_hip.h), signature records."""
        out = np.zeros(4, np.float64)
        self._lib.fd_verify_hip_tile_ingest_stats(self.tile, out.ctypes.data)
        return {"ms": float(out[0]), "frags": int(out[1]), "bytes": float(out[2]), "records": int(out[3])}

    def hist_init(self, min_ns, max_ns):
        """Reset both batch latency histograms with fd_histf edges over [min_ns, max_ns)."""
        if self._lib.fd_verify_hip_tile_hist_init(self.tile, int(min_ns), int(max_ns)):
            raise ValueError("max_ns must exceed min_ns")

    def hist(self, which="gpu"):
        """Batch latency histogram ("gpu" or "host"): counts, left edges (ns), sum (ns)."""
        counts = np.zeros(HIST_BUCKET_CNT, np.uint64)
        edge = np.zeros(HIST_BUCKET_CNT, np.uint64)
        total = np.zeros(1, np.uint64)
        w = {"gpu": 0, "host": 1}[which]
        self._lib.fd_verify_hip_tile_hist(self.tile, w, counts.ctypes.data, edge.ctypes.data, total.ctypes.data)
        return {"counts": counts, "left_edge_ns": edge, "sum_ns": int(total[0])}

    def close(self):
        if self.tile:
            self._lib.fd_verify_hip_tile_delete(self.tile)
            self.tile = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
