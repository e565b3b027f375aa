"""Batched SHA-512 on the GPU (C ABI: include/fd_sha512_hip.h, same library as
ed25519.py).

Reference interface mirrored: the multi-message batching API of
src/ballet/sha512/fd_sha512.h:232-419 (fd_sha512_batch_init / _add / _fini /
_abort; the AVX-512 build hashes 8 messages per call).  Here:

  sha512_batch_dev(verifier, n, pool, off, sz, out)   messages resident in HBM
  Sha512Batch(verifier).add(data) ... .fini()         host memory, the
                                                      reference's call shape
  sha512_many(list_of_bytes)                          convenience wrapper

There is no CPU fallback: a missing library raises.
"""
import ctypes

import numpy as np

from .ed25519 import _ptr, lib as _ed_lib

# Every symbol include/fd_sha512_hip.h declares (checked by tests/test_abi.py).
EXPORTS = ("fd_sha512_hip_batch_dev", "fd_sha512_hip_batch_align", "fd_sha512_hip_batch_footprint",
           "fd_sha512_hip_batch_init", "fd_sha512_hip_batch_add", "fd_sha512_hip_batch_fini",
           "fd_sha512_hip_batch_abort")

BATCH_MAX = 4096            # FD_SHA512_HIP_BATCH_MAX
MSG_MAX = 1 << 31           # FD_SHA512_HIP_MSG_MAX

_bound = False


def lib():
    global _bound
    L = _ed_lib()
    if not _bound:
        c = ctypes
        vp, u64 = c.c_void_p, c.c_ulong
        L.fd_sha512_hip_batch_dev.restype = c.c_int
        L.fd_sha512_hip_batch_dev.argtypes = [vp, u64, vp, vp, vp, vp, vp]
        L.fd_sha512_hip_batch_align.restype = u64
        L.fd_sha512_hip_batch_footprint.restype = u64
        L.fd_sha512_hip_batch_init.restype = vp
        L.fd_sha512_hip_batch_init.argtypes = [vp, vp]
        L.fd_sha512_hip_batch_add.restype = vp
        L.fd_sha512_hip_batch_add.argtypes = [vp, vp, u64, vp]
        L.fd_sha512_hip_batch_fini.restype = vp
        L.fd_sha512_hip_batch_fini.argtypes = [vp]
        L.fd_sha512_hip_batch_abort.restype = vp
        L.fd_sha512_hip_batch_abort.argtypes = [vp]
        _bound = True
    return L


def sha512_batch_dev(verifier, n, pool, off, sz, out, stream=None):
    """SHA-512 of n messages pool[off[i], +sz[i]) -> out (64 bytes each), all
    GPU tensors on the verifier's device; asynchronous on `stream` (the
    Verifier's stream= conventions).  pool must be readable up to the 16-byte
    boundary after each message."""
    n = int(n)
    L = lib()
    args = (verifier.ctx, n, _ptr(pool, 1, "pool", verifier.device), _ptr(off, 4 * n, "off", verifier.device),
            _ptr(sz, 4 * n, "sz", verifier.device), _ptr(out, 64 * n, "out", verifier.device))
    with verifier._stream(stream) as h:
        return L.fd_sha512_hip_batch_dev(*args, h)


class Sha512Batch:
    """fd_sha512_batch_t shape over host memory: add(data) returns a 64-byte
    bytearray that holds the digest once the batch has been flushed (by add
    when BATCH_MAX records are pending, or by fini).  verifier None: the
    process-wide context of the fd_ed25519_verify drop-in."""

    def __init__(self, verifier=None):
        L = lib()
        self._align = int(L.fd_sha512_hip_batch_align())
        fp = int(L.fd_sha512_hip_batch_footprint())
        self._mem = ctypes.create_string_buffer(fp + self._align)
        base = ctypes.addressof(self._mem)
        self._addr = (base + self._align - 1) // self._align * self._align
        self._keep = []
        self._b = L.fd_sha512_hip_batch_init(self._addr, verifier.ctx if verifier is not None else None)

    def add(self, data):
        data = bytes(data)
        if len(data) > MSG_MAX:
            raise ValueError("message longer than FD_SHA512_HIP_MSG_MAX")
        src = ctypes.create_string_buffer(data, max(len(data), 1))
        dst = ctypes.create_string_buffer(64)
        self._keep.append((src, dst))                       # readable until the flush
        lib().fd_sha512_hip_batch_add(self._b, ctypes.addressof(src), len(data), ctypes.addressof(dst))
        return dst

    def fini(self):
        lib().fd_sha512_hip_batch_fini(self._b)
        out = [bytes(d.raw) for _, d in self._keep]
        self._keep = []
        return out

    def abort(self):
        lib().fd_sha512_hip_batch_abort(self._b)
        self._keep = []


def sha512_many(messages, verifier=None):
    """Digests of a list of byte strings through the host batching API."""
    b = Sha512Batch(verifier)
    for m in messages:
        b.add(m)
    return b.fini()
