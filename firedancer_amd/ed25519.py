"""Host-side mirror of the reference's ed25519 verify interface, backed by the
gfx950 engine (firedancer_amd/libfd_ed25519_hip.so, C ABI in
include/fd_ed25519_hip.h).

Names, argument meaning and result codes follow src/ballet/ed25519/fd_ed25519.h
(fd_ed25519_verify :96-101, fd_ed25519_verify_batch_single_msg :124-130,
fd_ed25519_strerror :137-138).  There is no CPU fallback: if the HIP library is
missing or no GPU is present, every entry point raises.
"""
import contextlib
import ctypes
import os
import sys

import numpy as np

from .build import LIB, variant_path

FD_ED25519_SUCCESS = 0
FD_ED25519_ERR_SIG = -1
FD_ED25519_ERR_PUBKEY = -2
FD_ED25519_ERR_MSG = -3

ERRMODE_AVX512 = 0
ERRMODE_REF = 1

# Every symbol include/fd_ed25519_hip.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "fd_ed25519_verify", "fd_ed25519_verify_batch_single_msg", "fd_ed25519_strerror",
    "fd_ed25519_hip_ctx_new", "fd_ed25519_hip_ctx_delete", "fd_ed25519_hip_ctx_device",
    "fd_ed25519_hip_ctx_stream", "fd_ed25519_hip_ctx_reserve", "fd_ed25519_hip_set_errmode", "fd_ed25519_hip_verify_dev",
    "fd_ed25519_hip_verify_fixed_dev", "fd_ed25519_hip_verify_dev_count",
    "fd_ed25519_hip_verify_host", "fd_ed25519_hip_group_reduce_dev", "fd_ed25519_hip_sign_dev",
    "fd_ed25519_hip_sync", "fd_ed25519_hip_set_timing", "fd_ed25519_hip_get_timing",
    "fd_ed25519_hip_get_dsm_units", "fd_ed25519_hip_set_halfsize", "fd_ed25519_hip_test_halfsize",
    "fd_ed25519_hip_test_sha512", "fd_ed25519_hip_host_alloc", "fd_ed25519_hip_host_free",
    "fd_ed25519_hip_stage_async", "fd_ed25519_hip_test_prim", "fd_ed25519_hip_set_small_batch",
    "fd_ed25519_hip_dropin_init", "fd_ed25519_hip_dropin_stats", "fd_ed25519_hip_host_register",
    "fd_ed25519_hip_host_unregister", "fd_ed25519_hip_device_cnt", "fd_ed25519_hip_set_dsm_share",
    "fd_ed25519_hip_set_lat_cus", "fd_ed25519_hip_ctx_set_cu_mask", "fd_ed25519_hip_ctx_set_dsm_reserve",
)

_lib = None


def lib():
    """Load the engine library (raises if it was not built)."""
    global _lib
    if _lib is None:
        path = LIB
        v = os.environ.get("FD_ED25519_HIP_LIB")
        if v:   # an experimental build variant (firedancer_amd/build.py <variant> ...)
            path = v if os.sep in v else variant_path(v)
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build() (no CPU fallback exists)")
        # torch (device memory, streams) ships its own libamdhip64.so.7 with the
        # same soname as the system runtime this library links: whichever loads
        # first serves the whole process.  Load torch's first, always, so the
        # engine and torch share one runtime in every process and test order
        # (loaded the other way round, torch's CUDA init could fail afterwards).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(path)
        c = ctypes
        vp, u64 = c.c_void_p, c.c_ulong
        L.fd_ed25519_verify.restype = c.c_int
        L.fd_ed25519_verify.argtypes = [c.c_char_p, u64, c.c_char_p, c.c_char_p, vp]
        L.fd_ed25519_verify_batch_single_msg.restype = c.c_int
        L.fd_ed25519_verify_batch_single_msg.argtypes = [c.c_char_p, u64, c.c_char_p, c.c_char_p, vp, c.c_ubyte]
        L.fd_ed25519_strerror.restype = c.c_char_p
        L.fd_ed25519_strerror.argtypes = [c.c_int]
        L.fd_ed25519_hip_dropin_init.restype = c.c_int
        L.fd_ed25519_hip_dropin_init.argtypes = [c.c_int]
        L.fd_ed25519_hip_dropin_stats.argtypes = [c.POINTER(u64)]
        L.fd_ed25519_hip_ctx_new.restype = vp
        L.fd_ed25519_hip_ctx_new.argtypes = [c.c_int, u64]
        L.fd_ed25519_hip_ctx_delete.argtypes = [vp]
        L.fd_ed25519_hip_ctx_device.restype = c.c_int
        L.fd_ed25519_hip_ctx_device.argtypes = [vp]
        L.fd_ed25519_hip_ctx_stream.restype = vp
        L.fd_ed25519_hip_ctx_stream.argtypes = [vp]
        L.fd_ed25519_hip_set_errmode.argtypes = [vp, c.c_int]
        L.fd_ed25519_hip_set_halfsize.argtypes = [vp, c.c_int]
        L.fd_ed25519_hip_set_small_batch.argtypes = [vp, u64]
        L.fd_ed25519_hip_set_dsm_share.argtypes = [vp, u64]
        L.fd_ed25519_hip_set_lat_cus.argtypes = [vp, u64]
        L.fd_ed25519_hip_ctx_set_dsm_reserve.restype = c.c_int
        L.fd_ed25519_hip_ctx_set_dsm_reserve.argtypes = [vp, u64]
        L.fd_ed25519_hip_ctx_set_cu_mask.restype = c.c_int
        L.fd_ed25519_hip_ctx_set_cu_mask.argtypes = [vp, vp, c.c_uint]
        L.fd_ed25519_hip_test_halfsize.argtypes = [vp, c.c_ulong, vp, vp, vp]
        L.fd_ed25519_hip_test_sha512.argtypes = [vp, c.c_ulong, vp, vp, vp, vp, vp]
        L.fd_ed25519_hip_test_prim.restype = c.c_int
        L.fd_ed25519_hip_test_prim.argtypes = [vp, c.c_int, c.c_ulong, vp, vp, vp]
        L.fd_ed25519_hip_ctx_reserve.argtypes = [vp, u64]
        L.fd_ed25519_hip_host_alloc.restype = vp
        L.fd_ed25519_hip_host_alloc.argtypes = [u64]
        L.fd_ed25519_hip_host_free.argtypes = [vp]
        L.fd_ed25519_hip_stage_async.restype = c.c_int
        L.fd_ed25519_hip_stage_async.argtypes = [vp, vp, vp, u64, vp]
        L.fd_ed25519_hip_verify_dev.restype = c.c_int
        L.fd_ed25519_hip_verify_dev.argtypes = [vp, u64, vp, vp, vp, vp, vp, vp, vp, vp]
        L.fd_ed25519_hip_verify_fixed_dev.restype = c.c_int
        L.fd_ed25519_hip_verify_fixed_dev.argtypes = [vp, u64, vp, vp, vp, c.c_uint, vp, vp, vp]
        L.fd_ed25519_hip_verify_dev_count.restype = c.c_int
        L.fd_ed25519_hip_verify_dev_count.argtypes = [vp, u64, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.fd_ed25519_hip_verify_host.restype = c.c_int
        L.fd_ed25519_hip_verify_host.argtypes = [vp, u64, vp, vp, vp, u64, vp, vp, vp, vp]
        L.fd_ed25519_hip_group_reduce_dev.restype = c.c_int
        L.fd_ed25519_hip_group_reduce_dev.argtypes = [vp, u64, vp, vp, vp, vp, vp]
        L.fd_ed25519_hip_sign_dev.restype = c.c_int
        L.fd_ed25519_hip_sign_dev.argtypes = [vp, u64, vp, vp, vp, vp, vp, vp, vp]
        L.fd_ed25519_hip_set_timing.argtypes = [vp, c.c_int]
        L.fd_ed25519_hip_get_timing.argtypes = [vp, c.POINTER(c.c_double), c.POINTER(c.c_double), c.POINTER(u64)]
        L.fd_ed25519_hip_get_dsm_units.restype = u64
        L.fd_ed25519_hip_get_dsm_units.argtypes = [vp]
        L.fd_ed25519_hip_sync.restype = c.c_int
        L.fd_ed25519_hip_sync.argtypes = [vp]
        _lib = L
    return _lib


class HostBuffer:
    """Pinned, device-mapped host memory (fd_ed25519_hip_host_alloc): .array is
    a numpy uint8 view for the host, .ptr the address kernels use in place."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        self.ptr = lib().fd_ed25519_hip_host_alloc(self.nbytes)
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(self.nbytes, 1)).from_address(self.ptr))

    def close(self):
        if self.ptr:
            self.array = None
            lib().fd_ed25519_hip_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fd_ed25519_verify(msg, sig, public_key, sha=None):
    """fd_ed25519_user.c:135-230 semantics; returns an FD_ED25519_* code."""
    assert len(sig) == 64 and len(public_key) == 32
    return lib().fd_ed25519_verify(bytes(msg), len(msg), bytes(sig), bytes(public_key), None)


def fd_ed25519_verify_batch_single_msg(msg, signatures, pubkeys, batch_sz, shas=None):
    """fd_ed25519_user.c:232-310 semantics (batch_sz 0 or > 16 -> ERR_SIG)."""
    n = int(batch_sz)
    sigs = bytes(signatures) if n else b"\0" * 64
    pubs = bytes(pubkeys) if n else b"\0" * 32
    assert n > 16 or n == 0 or (len(sigs) >= 64 * n and len(pubs) >= 32 * n)
    return lib().fd_ed25519_verify_batch_single_msg(bytes(msg), len(msg), sigs, pubs, None, n & 0xff if n <= 255 else 255)


def fd_ed25519_strerror(err):
    return lib().fd_ed25519_strerror(int(err)).decode()


def fd_ed25519_hip_dropin_init(device=0):
    """Create the drop-in's process-wide context now (a tile's
    privileged_init); 0, or -1 if it exists on another device."""
    return lib().fd_ed25519_hip_dropin_init(int(device))


def dropin_stats():
    """(launches, calls served) of the drop-in's combining staging ring."""
    out = (ctypes.c_ulong * 2)()
    lib().fd_ed25519_hip_dropin_stats(out)
    return int(out[0]), int(out[1])


def _ptr(a, nbytes=0, name="buffer", device=None):
    """Device pointer of a GPU tensor for a *_dev entry point.  A host array
    would reach a GPU kernel as an unmapped address (a fault that can take the
    device down), and a tensor shorter than the records it is called for
    would be read out of bounds: both raise here instead.  A plain int is
    taken as a raw device pointer (the caller vouches for it)."""
    if a is None:
        return None
    if isinstance(a, int):
        return a
    if isinstance(a, np.ndarray) or not getattr(a, "is_cuda", False):
        raise TypeError(f"{name}: a GPU tensor is required (host data goes through verify_host)")
    if not a.is_contiguous():
        raise ValueError(f"{name}: tensor must be contiguous")
    if device is not None and a.device.index != device:
        raise ValueError(f"{name}: tensor on cuda:{a.device.index}, context on cuda:{device}")
    have = a.numel() * a.element_size()
    if have < nbytes:
        raise ValueError(f"{name}: {have} bytes, {nbytes} needed")
    return a.data_ptr()


CTX_STREAM = "ctx"   # stream= value naming the context's own (private) HIP stream


class Verifier:
    """One GPU context (device, stream, base-point table, chunk scratch).

    Stream of the *_dev calls: by default torch's current stream on the
    context's device, so a call is ordered after the torch work that produced
    its inputs and before the torch work that reads its outputs.  Pass
    stream=CTX_STREAM for the context's private stream (callers that keep
    several contexts in flight, and order them against torch themselves), or
    a raw hipStream_t handle (int).  Calls on one context are ordered among
    themselves whatever streams they name (fd_ed25519_hip.h)."""

    def __init__(self, device=0, chunk_sigs=1 << 20, errmode=ERRMODE_AVX512):
        self._lib = lib()
        self.ctx = self._lib.fd_ed25519_hip_ctx_new(int(device), int(chunk_sigs))
        if not self.ctx:
            raise RuntimeError("fd_ed25519_hip_ctx_new failed")
        self.device = int(device)
        self.set_errmode(errmode)

    def set_errmode(self, errmode):
        self._lib.fd_ed25519_hip_set_errmode(self.ctx, int(errmode))

    @property
    def stream(self):
        return self._lib.fd_ed25519_hip_ctx_stream(self.ctx)

    def close(self):
        if self.ctx:
            self._lib.fd_ed25519_hip_ctx_delete(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- host memory -------------------------------------------------------
    def verify_host(self, sigs, pubs, pool, msg_off, msg_sz):
        sigs = np.ascontiguousarray(sigs, np.uint8).reshape(-1, 64)
        n = sigs.shape[0]
        pubs = np.ascontiguousarray(pubs, np.uint8).reshape(n, 32)
        pool = np.ascontiguousarray(pool, np.uint8).reshape(-1)
        if pool.size == 0:
            pool = np.zeros(1, np.uint8)
        msg_off = np.ascontiguousarray(msg_off, np.uint32).reshape(n)
        msg_sz = np.ascontiguousarray(msg_sz, np.uint32).reshape(n)
        if n and int((msg_off.astype(np.uint64) + msg_sz).max()) > pool.size:
            raise ValueError("message outside the pool")
        codes = np.zeros(n, np.int8)
        bitmap = np.zeros((n + 63) // 64, np.uint64)
        if n:
            self._lib.fd_ed25519_hip_verify_host(self.ctx, n, sigs.ctypes.data, pubs.ctypes.data, pool.ctypes.data,
                                                 pool.size, msg_off.ctypes.data, msg_sz.ctypes.data,
                                                 codes.ctypes.data, bitmap.ctypes.data)
        return codes, bitmap

    # ---- device memory (torch tensors or raw pointers) ---------------------
    def _p(self, a, nbytes=0, name="buffer"):
        return _ptr(a, nbytes, name, self.device)

    @contextlib.contextmanager
    def _stream(self, stream):
        """Resolve a stream= argument to the hipStream_t handle passed to the C
        ABI (None = the context's stream).  Default (None): torch's current
        stream.  The C ABI reads a NULL handle as "the context's stream", so
        torch's legacy default stream (handle 0) cannot be named directly: the
        call then runs on the context's stream, forked from and joined back to
        torch's stream with events (the context stream is non-blocking, so
        without this nothing would order it against torch's work)."""
        if stream == CTX_STREAM:
            yield None
            return
        if stream is not None:
            yield int(stream)
            return
        torch = sys.modules.get("torch")
        if torch is None or not torch.cuda.is_available():
            yield None
            return
        cur = torch.cuda.current_stream(self.device)
        if cur.cuda_stream:
            yield cur.cuda_stream
            return
        ctx_s = torch.cuda.ExternalStream(self.stream, device=torch.device("cuda", self.device))
        fork = torch.cuda.Event()
        fork.record(cur)
        ctx_s.wait_event(fork)
        yield None
        join = torch.cuda.Event()
        join.record(ctx_s)
        cur.wait_event(join)

    def verify_dev(self, n, sigs, pubs, pool, msg_off, msg_sz, codes, bitmap=None, stream=None):
        """Message i = pool[msg_off[i], +msg_sz[i]).  The pool must stay
        readable 16 bytes past its last message byte: the caller guarantees
        it (checking it here would need the offsets on the host)."""
        n = int(n)
        args = (self.ctx, n, self._p(sigs, 64 * n, "sigs"), self._p(pubs, 32 * n, "pubs"), self._p(pool, 1, "pool"),
                self._p(msg_off, 4 * n, "msg_off"), self._p(msg_sz, 4 * n, "msg_sz"), self._p(codes, n, "codes"),
                self._p(bitmap, 8 * ((n + 63) // 64), "bitmap"))
        with self._stream(stream) as h:
            return self._lib.fd_ed25519_hip_verify_dev(*args, h)

    def verify_dev_count(self, n_max, d_n, sigs, pubs, pool, msg_off, msg_sz, codes, bitmap=None, stream=None):
        """verify_dev with the record count in device memory (uint32 *d_n)."""
        n = int(n_max)
        args = (self.ctx, n, self._p(d_n, 4, "d_n"), self._p(sigs, 64 * n, "sigs"), self._p(pubs, 32 * n, "pubs"),
                self._p(pool, 1, "pool"), self._p(msg_off, 4 * n, "msg_off"), self._p(msg_sz, 4 * n, "msg_sz"),
                self._p(codes, n, "codes"), self._p(bitmap, 8 * ((n + 63) // 64), "bitmap"))
        with self._stream(stream) as h:
            return self._lib.fd_ed25519_hip_verify_dev_count(*args, h)

    def verify_fixed_dev(self, n, sigs, pubs, msgs, msg_sz, codes, bitmap=None, stream=None):
        """Fixed-size messages back to back: message i = msgs[i*msg_sz, (i+1)*msg_sz);
        msgs must hold 16 readable bytes past the last message."""
        n = int(n)
        args = (self.ctx, n, self._p(sigs, 64 * n, "sigs"), self._p(pubs, 32 * n, "pubs"),
                self._p(msgs, n * int(msg_sz) + 16, "msgs (+16 readable bytes)"), int(msg_sz),
                self._p(codes, n, "codes"), self._p(bitmap, 8 * ((n + 63) // 64), "bitmap"))
        with self._stream(stream) as h:
            return self._lib.fd_ed25519_hip_verify_fixed_dev(*args, h)

    def group_reduce_dev(self, n_groups, first, cnt, sig_codes, group_codes, stream=None):
        ng = int(n_groups)
        args = (self.ctx, ng, self._p(first, 4 * ng, "first"), self._p(cnt, ng, "cnt"),
                self._p(sig_codes, 1, "sig_codes"), self._p(group_codes, ng, "group_codes"))
        with self._stream(stream) as h:
            return self._lib.fd_ed25519_hip_group_reduce_dev(*args, h)

    def sign_dev(self, n, prvs, pool, msg_off, msg_sz, pubs, sigs, stream=None):
        n = int(n)
        args = (self.ctx, n, self._p(prvs, 32 * n, "prvs"), self._p(pool, 1, "pool"), self._p(msg_off, 4 * n, "msg_off"),
                self._p(msg_sz, 4 * n, "msg_sz"), self._p(pubs, 32 * n, "pubs"), self._p(sigs, 64 * n, "sigs"))
        with self._stream(stream) as h:
            return self._lib.fd_ed25519_hip_sign_dev(*args, h)

    def set_dsm_share(self, share):
        """k_verify_dsm grid = 1/share of the resident workgroup slots (contexts sharing the GPU)."""
        lib().fd_ed25519_hip_set_dsm_share(self.ctx, int(share))

    def set_halfsize(self, on):
        """Half-size scalars (default) or the full-length pair (k, 1): same verdicts."""
        self._lib.fd_ed25519_hip_set_halfsize(self.ctx, 1 if on else 0)

    def set_small_batch(self, max_n):
        """Calls of at most max_n records take the latency kernel (0: never)."""
        self._lib.fd_ed25519_hip_set_small_batch(self.ctx, int(max_n))

    def set_cu_mask(self, cus=None):
        """Run the context's stream on the listed CU indices only (None: all)."""
        if not cus:
            return self._lib.fd_ed25519_hip_ctx_set_cu_mask(self.ctx, None, 0)
        words = (max(cus) // 32) + 1
        m = np.zeros(words, np.uint32)
        for c_ in cus:
            m[c_ // 32] |= np.uint32(1 << (c_ % 32))
        self._m = m
        return self._lib.fd_ed25519_hip_ctx_set_cu_mask(self.ctx, m.ctypes.data, words)

    def set_lat_cus(self, cus):
        """k_verify_lat workgroup slots a latency-path call may fill with racing copies (1: one copy)."""
        self._lib.fd_ed25519_hip_set_lat_cus(self.ctx, int(cus))

    def test_halfsize(self, n, d_k, d_out, stream=None):
        """Test hook: device half-size reduction (see fd_ed25519_hip_test_halfsize)."""
        n = int(n)
        args = (self.ctx, n, self._p(d_k, 32 * n, "k"), self._p(d_out, 72 * n, "out"))
        with self._stream(stream) as h:
            return self._lib.fd_ed25519_hip_test_halfsize(*args, h)

    def test_sha512(self, n, pool, msg_off, msg_sz, out, stream=None):
        """Test hook: device SHA-512 of n messages -> out (128 bytes each: the
        per-lane path's digests, then the cooperative LDS path's)."""
        n = int(n)
        args = (self.ctx, n, self._p(pool, 1, "pool"), self._p(msg_off, 4 * n, "msg_off"),
                self._p(msg_sz, 4 * n, "msg_sz"), self._p(out, 128 * n, "out"))
        with self._stream(stream) as h:
            return self._lib.fd_ed25519_hip_test_sha512(*args, h)

    def test_prim(self, op, n, d_in, d_out, stream=None):
        """Test hook: one device primitive (FD_ED25519_HIP_PRIM_*, see
        fd_ed25519_hip_test_prim) over n items of 32 u32 words in and out."""
        n = int(n)
        args = (self.ctx, int(op), n, self._p(d_in, 128 * n, "in"), self._p(d_out, 128 * n, "out"))
        with self._stream(stream) as h:
            rc = self._lib.fd_ed25519_hip_test_prim(*args, h)
        if rc:
            raise ValueError(f"test_prim: unknown op {op}")
        return rc

    def stage_async(self, d_dst, h_src, nbytes, stream=None):
        """Host -> device copy of nbytes (h_src: a HostBuffer or raw host address) on a stream."""
        src = h_src.ptr if isinstance(h_src, HostBuffer) else int(h_src)
        with self._stream(stream) as h:
            return self._lib.fd_ed25519_hip_stage_async(self.ctx, self._p(d_dst, int(nbytes), "d_dst"), src,
                                                        int(nbytes), h)

    def set_timing(self, on):
        self._lib.fd_ed25519_hip_set_timing(self.ctx, 1 if on else 0)

    def get_timing(self):
        """(prep_ms, dsm_ms, launches) accumulated since set_timing()."""
        a, b, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_ulong()
        self._lib.fd_ed25519_hip_get_timing(self.ctx, ctypes.byref(a), ctypes.byref(b), ctypes.byref(n))
        return a.value, b.value, n.value

    def get_dsm_units(self):
        """Signatures that ran through k_verify_dsm while timing was on."""
        return int(self._lib.fd_ed25519_hip_get_dsm_units(self.ctx))

    def sync(self):
        self._lib.fd_ed25519_hip_sync(self.ctx)
