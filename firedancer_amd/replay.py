"""Host-side mirror of the bulk verify callers outside the verify tile, backed
by the gfx950 engine (C ABI: include/fd_replay_hip.h, same library as
ed25519.py).

Reference interfaces mirrored:
  fd_executor_txn_verify   src/flamenco/runtime/fd_executor.c:1607-1623
                           (FD_RUNTIME_EXECUTE_SUCCESS / FD_RUNTIME_TXN_ERR_
                           SIGNATURE_FAILURE, fd_runtime_err.h:4,19), called
                           per txn by the exec tile (fd_exec_tile.c:161)
  FEC-set root check       src/disco/shred/fd_fec_resolver.c:476
                           (fd_ed25519_verify of a 32-B Merkle root)
  fd_precompile_ed25519_verify
                           src/flamenco/runtime/program/fd_precompiles.c:114-211
                           (ed25519 program instructions: offset records naming
                           signature / pubkey / message spans, possibly in
                           other instructions of the txn)

Both take whole batches (a block's transactions, a poll's FEC sets) in device
memory.  There is no CPU fallback.
"""
import ctypes

import numpy as np

from .ed25519 import _ptr, lib as _ed_lib

FD_RUNTIME_EXECUTE_SUCCESS = 0
FD_RUNTIME_TXN_ERR_SIGNATURE_FAILURE = -13

# Every symbol include/fd_replay_hip.h declares (checked by tests/test_abi.py).
EXPORTS = ("fd_replay_hip_new", "fd_replay_hip_delete", "fd_replay_hip_txn_verify_dev", "fd_replay_hip_poll",
           "fd_replay_hip_txn_verify_host", "fd_replay_hip_wait",
           "fd_fec_hip_verify_roots_dev", "fd_precompile_hip_new", "fd_precompile_hip_delete",
           "fd_precompile_hip_ed25519_verify_dev")

# fd_executor_err.h:14,40 and fd_precompiles.h:16-18
FD_EXECUTOR_INSTR_SUCCESS = 0
FD_EXECUTOR_INSTR_ERR_CUSTOM_ERR = -26
FD_EXECUTOR_PRECOMPILE_ERR_SIGNATURE = 2
FD_EXECUTOR_PRECOMPILE_ERR_DATA_OFFSET = 3
FD_EXECUTOR_PRECOMPILE_ERR_INSTR_DATA_SIZE = 4
PRECOMPILE_SIG_MAX = 87
PRECOMPILE_DATA_MAX = 1232

# fd_precompile_hip_desc_t / fd_precompile_hip_instr_t (include/fd_replay_hip.h)
PC_DESC_DTYPE = np.dtype([("data_off", "<u4"), ("data_sz", "<u2"), ("instr_cnt", "<u2"), ("instr_base", "<u4"),
                          ("_pad", "<u4")])
PC_INSTR_DTYPE = np.dtype([("data_off", "<u4"), ("data_sz", "<u4")])
assert PC_DESC_DTYPE.itemsize == 16 and PC_INSTR_DTYPE.itemsize == 8

# fd_txn_hip_desc_t (16 bytes): the fd_txn_p_t payload span and the fd_txn_t
# fields fd_executor_txn_verify reads (fd_txn.h:186-249)
DESC_DTYPE = np.dtype([("payload_off", "<u4"), ("payload_sz", "<u2"), ("signature_off", "<u2"),
                       ("message_off", "<u2"), ("acct_addr_off", "<u2"), ("signature_cnt", "u1"),
                       ("_pad", "u1", (3,))])
assert DESC_DTYPE.itemsize == 16

_bound = False


def lib():
    global _bound
    L = _ed_lib()
    if not _bound:
        c = ctypes
        vp, u64 = c.c_void_p, c.c_ulong
        L.fd_replay_hip_new.restype = vp
        L.fd_replay_hip_new.argtypes = [vp, u64]
        L.fd_replay_hip_delete.argtypes = [vp]
        L.fd_replay_hip_txn_verify_dev.restype = c.c_int
        L.fd_replay_hip_txn_verify_dev.argtypes = [vp, u64, vp, vp, vp, vp]
        L.fd_replay_hip_poll.restype = c.c_int
        L.fd_replay_hip_poll.argtypes = [vp]
        L.fd_replay_hip_txn_verify_host.restype = c.c_int
        L.fd_replay_hip_txn_verify_host.argtypes = [vp, u64, vp, u64, vp, vp, vp]
        L.fd_replay_hip_wait.restype = c.c_int
        L.fd_replay_hip_wait.argtypes = [vp]
        L.fd_fec_hip_verify_roots_dev.restype = c.c_int
        L.fd_fec_hip_verify_roots_dev.argtypes = [vp, u64, vp, vp, vp, vp, vp]
        L.fd_precompile_hip_new.restype = vp
        L.fd_precompile_hip_new.argtypes = [vp, u64]
        L.fd_precompile_hip_delete.argtypes = [vp]
        L.fd_precompile_hip_ed25519_verify_dev.restype = c.c_int
        L.fd_precompile_hip_ed25519_verify_dev.argtypes = [vp, u64, vp, vp, vp, vp, vp, vp]
        _bound = True
    return L


def descs_from_txn_t(txn_t, payload_off, payload_sz):
    """fd_txn_hip_desc_t records from fd_txn_t bytes (one row per txn: byte 1
    signature_cnt, 2-3 signature_off, 4-5 message_off, 10-11 acct_addr_off)."""
    t = np.ascontiguousarray(txn_t, np.uint8)
    d = np.zeros(t.shape[0], DESC_DTYPE)
    d["payload_off"] = payload_off
    d["payload_sz"] = payload_sz
    d["signature_cnt"] = t[:, 1]
    d["signature_off"] = t[:, 2].astype(np.uint16) | (t[:, 3].astype(np.uint16) << 8)
    d["message_off"] = t[:, 4].astype(np.uint16) | (t[:, 5].astype(np.uint16) << 8)
    d["acct_addr_off"] = t[:, 10].astype(np.uint16) | (t[:, 11].astype(np.uint16) << 8)
    return d


class ReplayVerifier:
    """fd_executor_txn_verify over batches of up to max_txn parsed txns."""

    def __init__(self, verifier, max_txn):
        self._lib = lib()
        self.verifier = verifier
        self.r = self._lib.fd_replay_hip_new(verifier.ctx, int(max_txn))
        if not self.r:
            raise RuntimeError("fd_replay_hip_new failed")
        self.max_txn = int(max_txn)

    def txn_verify_dev(self, n, pool, desc, result, stream=None):
        """pool: device bytes; desc: device fd_txn_hip_desc_t[n]; result: device int32[n]."""
        n, dev = int(n), self.verifier.device
        args = (self.r, n, _ptr(pool, 1, "pool", dev), _ptr(desc, 16 * n, "desc", dev),
                _ptr(result, 4 * n, "result", dev))
        with self.verifier._stream(stream) as h:
            rc = self._lib.fd_replay_hip_txn_verify_dev(*args, h)
        if rc:
            raise ValueError(f"fd_replay_hip_txn_verify_dev: n={n} > max_txn={self.max_txn}")

    def txn_verify_host(self, n, pool, desc, result, stream=None):
        """fd_replay_hip_txn_verify_host: pool / desc / result are host numpy
        arrays (uint8, DESC_DTYPE[n], int32[n]) that must stay alive and
        untouched until poll() == 1 or wait().  Raises on a rejected call."""
        n = int(n)
        for a, nm in ((pool, "pool"), (desc, "desc"), (result, "result")):
            if not (isinstance(a, np.ndarray) and a.flags.c_contiguous):
                raise TypeError(f"{nm}: contiguous numpy array required")
        if desc.dtype != DESC_DTYPE or desc.size < n or result.dtype != np.int32 or result.size < n:
            raise ValueError("desc must be DESC_DTYPE[n], result int32[n]")
        with self.verifier._stream(stream) as h:
            rc = self._lib.fd_replay_hip_txn_verify_host(self.r, n, pool.ctypes.data, pool.nbytes, desc.ctypes.data,
                                                          result.ctypes.data, h)
        if rc:
            raise ValueError(f"fd_replay_hip_txn_verify_host rejected n={n} pool_sz={pool.nbytes}")

    def poll(self):
        """fd_replay_hip_poll: 1 when the last txn_verify_dev / _host is done,
        0 while it runs, -1 before any call."""
        return self._lib.fd_replay_hip_poll(self.r)

    def wait(self):
        self._lib.fd_replay_hip_wait(self.r)

    def close(self):
        if self.r:
            self._lib.fd_replay_hip_delete(self.r)
            self.r = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fec_verify_roots_dev(verifier, n, roots, sigs, pubs, codes, stream=None):
    """FEC-set root check: codes[i] = fd_ed25519_verify(roots[32i:32i+32], sigs[i], pubs[i])."""
    n, dev = int(n), verifier.device
    args = (verifier.ctx, n, _ptr(roots, 32 * n + 16, "roots (+16 readable bytes)", dev),
            _ptr(sigs, 64 * n, "sigs", dev), _ptr(pubs, 32 * n, "pubs", dev), _ptr(codes, n, "codes", dev))
    with verifier._stream(stream) as h:
        return lib().fd_fec_hip_verify_roots_dev(*args, h)


class PrecompileVerifier:
    """fd_precompile_ed25519_verify over batches of up to max_instr ed25519
    program instructions (fd_precompile_hip_ed25519_verify_dev)."""

    def __init__(self, verifier, max_instr):
        self._lib = lib()
        self.verifier = verifier
        self.p = self._lib.fd_precompile_hip_new(verifier.ctx, int(max_instr))
        if not self.p:
            raise RuntimeError("fd_precompile_hip_new failed")
        self.max_instr = int(max_instr)

    def ed25519_verify_dev(self, n, pool, desc, instr_tab, err, custom_err, stream=None):
        """pool: device bytes (readable 16 bytes past the last span); desc:
        device PC_DESC_DTYPE[n]; instr_tab: device PC_INSTR_DTYPE[...];
        err: device int32[n]; custom_err: device uint32[n]."""
        n, dev = int(n), self.verifier.device
        args = (self.p, n, _ptr(pool, 1, "pool", dev), _ptr(desc, 16 * n, "desc", dev),
                _ptr(instr_tab, 8, "instr_tab", dev), _ptr(err, 4 * n, "err", dev),
                _ptr(custom_err, 4 * n, "custom_err", dev))
        with self.verifier._stream(stream) as h:
            rc = self._lib.fd_precompile_hip_ed25519_verify_dev(*args, h)
        if rc:
            raise ValueError(f"fd_precompile_hip_ed25519_verify_dev: n={n} > max_instr={self.max_instr}")

    def close(self):
        if self.p:
            self._lib.fd_precompile_hip_delete(self.p)
            self.p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
