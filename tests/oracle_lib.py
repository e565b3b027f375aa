"""ctypes binding to the CPU oracle (oracle/liboracle.so) -- test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ERRMODE_AVX512, ERRMODE_REF = 0, 1

_lib = None


def _u8p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "oracle"])
        L = ctypes.CDLL(path)
        c = ctypes
        L.oracle_verify.restype = c.c_int
        L.oracle_verify.argtypes = [c.c_char_p, c.c_size_t, c.c_char_p, c.c_char_p, c.c_int]
        L.oracle_verify_batch_single_msg.restype = c.c_int
        L.oracle_verify_batch_single_msg.argtypes = [c.c_char_p, c.c_size_t, c.c_char_p, c.c_char_p, c.c_uint, c.c_int]
        L.oracle_verify_many.argtypes = [c.c_size_t, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p,
                                         c.c_void_p, c.c_int]
        L.oracle_sign_many.argtypes = [c.c_size_t, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p]
        L.oracle_public_from_private.argtypes = [c.c_char_p, c.c_char_p]
        L.oracle_sign.argtypes = [c.c_char_p, c.c_char_p, c.c_size_t, c.c_char_p, c.c_char_p]
        L.oracle_sha512.argtypes = [c.c_char_p, c.c_char_p, c.c_size_t]
        L.oracle_hram.argtypes = [c.c_char_p, c.c_char_p, c.c_char_p, c.c_char_p, c.c_size_t]
        L.oracle_scalar_reduce.argtypes = [c.c_char_p, c.c_char_p]
        L.oracle_point_decode.restype = c.c_int
        L.oracle_point_decode.argtypes = [c.c_char_p, c.c_char_p]
        L.oracle_point_is_small_order.restype = c.c_int
        L.oracle_point_is_small_order.argtypes = [c.c_char_p]
        _lib = L
    return _lib


def verify(msg, sig, pub, errmode=ERRMODE_AVX512):
    return lib().oracle_verify(msg, len(msg), sig, pub, errmode)


def verify_batch_single_msg(msg, sigs, pubs, n, errmode=ERRMODE_AVX512):
    return lib().oracle_verify_batch_single_msg(msg, len(msg), sigs, pubs, n, errmode)


def verify_many(sigs, pubs, pool, msg_off, msg_sz, errmode=ERRMODE_AVX512):
    n = sigs.shape[0]
    sigs = np.ascontiguousarray(sigs, np.uint8); pubs = np.ascontiguousarray(pubs, np.uint8)
    pool = np.ascontiguousarray(pool, np.uint8)
    if pool.size == 0:
        pool = np.zeros(1, np.uint8)
    msg_off = np.ascontiguousarray(msg_off, np.uint32); msg_sz = np.ascontiguousarray(msg_sz, np.uint32)
    codes = np.zeros(n, np.int8)
    lib().oracle_verify_many(n, sigs.ctypes.data, pubs.ctypes.data, pool.ctypes.data, msg_off.ctypes.data,
                             msg_sz.ctypes.data, codes.ctypes.data, errmode)
    return codes


def sign_many(prvs, pool, msg_off, msg_sz):
    n = prvs.shape[0]
    prvs = np.ascontiguousarray(prvs, np.uint8)
    pool = np.ascontiguousarray(pool, np.uint8)
    if pool.size == 0:
        pool = np.zeros(1, np.uint8)
    msg_off = np.ascontiguousarray(msg_off, np.uint32); msg_sz = np.ascontiguousarray(msg_sz, np.uint32)
    pubs = np.zeros((n, 32), np.uint8); sigs = np.zeros((n, 64), np.uint8)
    lib().oracle_sign_many(n, prvs.ctypes.data, pubs.ctypes.data, sigs.ctypes.data, pool.ctypes.data,
                           msg_off.ctypes.data, msg_sz.ctypes.data)
    return pubs, sigs


def sha512(data):
    out = ctypes.create_string_buffer(64)
    lib().oracle_sha512(out, data, len(data))
    return out.raw


def hram(R, A, msg):
    out = ctypes.create_string_buffer(32)
    lib().oracle_hram(out, R, A, msg, len(msg))
    return out.raw


def scalar_reduce(b64):
    out = ctypes.create_string_buffer(32)
    lib().oracle_scalar_reduce(out, b64)
    return out.raw


def public_from_private(prv):
    out = ctypes.create_string_buffer(32)
    lib().oracle_public_from_private(out, prv)
    return out.raw


def sign(msg, pub, prv):
    out = ctypes.create_string_buffer(64)
    lib().oracle_sign(out, msg, len(msg), pub, prv)
    return out.raw
