"""Synthetic ed25519-program (precompile) instructions for the parity tests of
fd_precompile_hip_ed25519_verify_dev, and a binding to the oracle's
restatement (oracle/fd_precompile_oracle.c) -- test infrastructure only.

Instruction data layout (fd_precompiles.c:114-211; the shape
new_ed25519_instruction builds): [sig_cnt, 0, sig_cnt x 14-byte offset
records, payload...], offset record = 7 little-endian u16: sig_offset,
sig_instr_idx, pubkey_offset, pubkey_instr_idx, msg_offset, msg_data_sz,
msg_instr_idx.  Index 0xFFFF names the instruction itself.
"""
import ctypes
import os
import struct

import numpy as np

import oracle_lib as O

PC_DESC = np.dtype([("data_off", "<u4"), ("data_sz", "<u2"), ("instr_cnt", "<u2"), ("instr_base", "<u4"),
                    ("_pad", "<u4")])
PC_INSTR = np.dtype([("data_off", "<u4"), ("data_sz", "<u4")])
CUR = 0xFFFF


def offsets(sig_off, sig_idx, pub_off, pub_idx, msg_off, msg_sz, msg_idx):
    return struct.pack("<7H", sig_off, sig_idx, pub_off, pub_idx, msg_off, msg_sz, msg_idx)


class Keys:
    def __init__(self, seed, n=8):
        rng = np.random.default_rng(seed)
        self.prv = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(n)]
        self.pub = [O.public_from_private(p) for p in self.prv]

    def sign(self, k, msg):
        return O.sign(msg, self.pub[k], self.prv[k])


def self_contained(keys, rng, nsig, bad=()):
    """One instruction carrying nsig (<= 5) (pubkey, signature, message)
    triples in its own data, offsets through index 0xFFFF; signatures listed
    in bad get one bit flipped.  Instruction data stays within the 1232-byte
    transaction MTU."""
    head = 2 + 14 * nsig
    body, recs = b"", []
    for i in range(nsig):
        k = int(rng.integers(0, len(keys.pub)))
        msg = rng.integers(0, 256, int(rng.integers(0, 120)), dtype=np.uint8).tobytes()   # <= 1232 B in all
        sig = bytearray(keys.sign(k, msg))
        if i in bad:
            sig[int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
        pub_at = head + len(body); body += keys.pub[k]
        sig_at = head + len(body); body += bytes(sig)
        msg_at = head + len(body); body += msg
        recs.append(offsets(sig_at, CUR, pub_at, CUR, msg_at, len(msg), CUR))
    return bytes([nsig, 0]) + b"".join(recs) + body


def cross_instruction(keys, rng, own_idx):
    """A two-instruction txn: instruction 0 holds the message, pubkey and
    signature; instruction 1 (the precompile) points into it by index."""
    k = int(rng.integers(0, len(keys.pub)))
    msg = rng.integers(0, 256, int(rng.integers(1, 300)), dtype=np.uint8).tobytes()
    other = b"\x07" * 5 + keys.pub[k] + keys.sign(k, msg) + msg
    data = bytes([1, 0]) + offsets(5 + 32, 0, 5, 0, 5 + 96, len(msg), 0)
    return [other, data], 1


def random_block(seed, n_instr, keys=None):
    """n_instr precompile instructions with every outcome class: valid
    (own-data and cross-instruction), bad signatures at random positions,
    offset records out of range or naming a missing instruction, size
    errors, the [0, 0] edge case.  Returns (pool, desc, tab) numpy arrays in
    the GPU entry's layout."""
    rng = np.random.default_rng(seed)
    keys = keys or Keys(seed)
    txns = []                                            # (list of instruction datas, precompile index)
    for _ in range(n_instr):
        r = rng.random()
        if r < 0.45:
            nsig = int(rng.integers(1, 6))
            bad = set(rng.choice(nsig, int(rng.integers(0, 2)), replace=False).tolist()) if rng.random() < 0.3 else ()
            txns.append(([b"\x01\x02", self_contained(keys, rng, nsig, bad)], 1))
        elif r < 0.6:
            txns.append(cross_instruction(keys, rng, 1))
        elif r < 0.7:                                    # an offset record past the data / a missing instruction
            d = bytearray(self_contained(keys, rng, int(rng.integers(1, 4))))
            i = int(rng.integers(0, d[0]))
            field = int(rng.integers(0, 7))
            val = int(rng.choice([0xFFF0, len(d), 2, 5, 0xFFFE]))
            d[2 + 14 * i + 2 * field: 4 + 14 * i + 2 * field] = struct.pack("<H", val)
            txns.append(([bytes(d)], 0))
        elif r < 0.8:                                    # size-class errors and edge cases
            c = int(rng.integers(0, 6))
            d = [b"\x00\x00", b"\x00", b"", b"\x01\x00", bytes(16), bytes([3, 0]) + bytes(30)][c]
            txns.append(([d], 0))
        elif r < 0.9:                                    # truncated: sig_cnt larger than the records present
            d = self_contained(keys, rng, 2)
            txns.append(([bytes([9]) + d[1:]], 0))
        else:                                            # bad signature then an offset error (order matters)
            d = bytearray(self_contained(keys, rng, 3, bad={int(rng.integers(0, 3))}))
            j = int(rng.integers(0, 3))
            d[2 + 14 * j + 2: 4 + 14 * j + 2] = struct.pack("<H", 7)    # sig_instr_idx 7: missing
            txns.append(([bytes(d)], 0))
    chunks, pos = [], 0
    tab, desc = [], np.zeros(len(txns), PC_DESC)
    for j, (datas, own) in enumerate(txns):
        base = len(tab)
        for d in datas:
            pos = (pos + 7) // 8 * 8 + int(rng.integers(0, 8))     # unaligned starts
            chunks.append((pos, d))
            tab.append((pos, len(d)))
            pos += len(d)
        desc[j]["data_off"], desc[j]["data_sz"] = tab[base + own]
        desc[j]["instr_cnt"] = len(datas)
        desc[j]["instr_base"] = base
    assert max(len(d) for _, d in chunks) <= 1232
    pool = np.zeros(pos + 16, np.uint8)
    for o, d in chunks:
        pool[o:o + len(d)] = np.frombuffer(d, np.uint8)
    return pool, desc, np.array(tab, PC_INSTR).reshape(-1)


_bound = False


def olib():
    global _bound
    L = O.lib()
    if not _bound:
        c = ctypes
        vp = c.c_void_p
        L.oracle_precompile_ed25519_verify.restype = c.c_int
        L.oracle_precompile_ed25519_verify.argtypes = [c.c_char_p, c.c_size_t, vp, vp, c.c_size_t,
                                                       c.POINTER(c.c_uint32)]
        L.oracle_precompile_ed25519_verify_many.argtypes = [c.c_size_t, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        _bound = True
    return L


def oracle_verify(data, instrs):
    """(err, custom_err) of fd_precompile_ed25519_verify for one instruction
    whose txn's instruction datas are instrs."""
    bufs = [ctypes.create_string_buffer(bytes(d), max(len(d), 1)) for d in instrs]
    ptrs = (ctypes.c_void_p * max(len(bufs), 1))(*[ctypes.addressof(b) for b in bufs])
    szs = (ctypes.c_size_t * max(len(bufs), 1))(*[len(d) for d in instrs])
    cur = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    ce = ctypes.c_uint32(0)
    err = olib().oracle_precompile_ed25519_verify(ctypes.cast(cur, ctypes.c_char_p), len(data), ptrs, szs,
                                                  len(instrs), ctypes.byref(ce))
    return err, ce.value


def oracle_many(pool, desc, tab):
    n = desc.size
    err = np.zeros(n, np.int32)
    ce = np.zeros(n, np.uint32)
    doff = np.ascontiguousarray(desc["data_off"]); dsz = np.ascontiguousarray(desc["data_sz"])
    icnt = np.ascontiguousarray(desc["instr_cnt"]); ibase = np.ascontiguousarray(desc["instr_base"])
    toff = np.ascontiguousarray(tab["data_off"]); tsz = np.ascontiguousarray(tab["data_sz"])
    olib().oracle_precompile_ed25519_verify_many(n, pool.ctypes.data, doff.ctypes.data, dsz.ctypes.data,
                                                 icnt.ctypes.data, ibase.ctypes.data, toff.ctypes.data,
                                                 tsz.ctypes.data, err.ctypes.data, ce.ctypes.data)
    return err, ce


_rlib = None


def ref_path():
    return os.path.join(O.ORACLE_DIR, "_ref", "libfdref_precompile.so")


def rlib():
    """The reference's own fd_precompile_ed25519_verify (fd_precompiles.c:120-222),
    compiled from its source by oracle/Makefile behind ref_precompile_drv.c."""
    global _rlib
    if _rlib is None:
        c = ctypes
        L = c.CDLL(ref_path())
        L.ref_precompile_ed25519_verify.restype = c.c_int
        L.ref_precompile_ed25519_verify.argtypes = [c.c_char_p, c.c_ulong, c.c_void_p, c.c_void_p, c.c_ulong,
                                                    c.POINTER(c.c_uint32)]
        _rlib = L
    return _rlib


def ref_verify(data, instrs):
    """(err, custom_err) from the reference itself, same arguments as oracle_verify."""
    bufs = [ctypes.create_string_buffer(bytes(d), max(len(d), 1)) for d in instrs]
    ptrs = (ctypes.c_void_p * max(len(bufs), 1))(*[ctypes.addressof(b) for b in bufs])
    szs = (ctypes.c_ulong * max(len(bufs), 1))(*[len(d) for d in instrs])
    cur = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    ce = ctypes.c_uint32(0)
    err = rlib().ref_precompile_ed25519_verify(ctypes.cast(cur, ctypes.c_char_p), len(data), ptrs, szs,
                                               len(instrs), ctypes.byref(ce))
    assert err != -1000, "driver refused the instruction (size or count past the context's arrays)"
    return err, ce.value


def ref_many(pool, desc, tab):
    """The reference over random_block's layout: (err, custom_err) arrays."""
    n = desc.size
    err = np.zeros(n, np.int32)
    ce = np.zeros(n, np.uint32)
    for j in range(n):
        b, k = int(desc[j]["instr_base"]), int(desc[j]["instr_cnt"])
        instrs = [pool[int(t["data_off"]):int(t["data_off"]) + int(t["data_sz"])].tobytes() for t in tab[b:b + k]]
        o, s = int(desc[j]["data_off"]), int(desc[j]["data_sz"])
        err[j], ce[j] = ref_verify(pool[o:o + s].tobytes(), instrs)
    return err, ce
