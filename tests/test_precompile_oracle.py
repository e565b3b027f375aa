"""CPU: the oracle's restatement of fd_precompile_ed25519_verify
(oracle/fd_precompile_oracle.c) on cases whose outcome follows directly from
the reference's source text (src/flamenco/runtime/program/fd_precompiles.c:
76-107 fetch rules, 114-211 instruction rules).  The same restatement is
pinned to the reference's own precompile, compiled from its source, in
tests/test_precompile_ref.py."""
import struct

import numpy as np

import precompile_lib as P

SUCCESS, CUSTOM = 0, -26
SIG, OFFSET, SIZE = 2, 3, 4


def one(keys, msg=b"hello", k=0, bad=False):
    sig = bytearray(keys.sign(k, msg))
    if bad:
        sig[5] ^= 4
    return keys.pub[k], bytes(sig), msg


def instr(triples, idx=P.CUR, head_extra=b""):
    head = 2 + 14 * len(triples)
    body, recs = head_extra, []
    for pub, sig, msg in triples:
        pa = head + len(body); body += pub
        sa = head + len(body); body += sig
        ma = head + len(body); body += msg
        recs.append(P.offsets(sa, idx, pa, idx, ma, len(msg), idx))
    return bytes([len(triples), 0]) + b"".join(recs) + body


def test_size_rules():
    # :130-141 the [0, 0] edge case succeeds; anything else under 16 bytes is a size error
    assert P.oracle_verify(b"\x00\x00", []) == (SUCCESS, 0)
    for d in (b"", b"\x00", b"\x01\x00", b"\x00\x00\x00", bytes(15)):
        assert P.oracle_verify(d, []) == (CUSTOM, SIZE), d
    # :143-147 zero signatures with >= 16 bytes
    assert P.oracle_verify(bytes(16), []) == (CUSTOM, SIZE)
    # :150-154 fewer bytes than sig_cnt offset records
    assert P.oracle_verify(bytes([3, 0]) + bytes(39), []) == (CUSTOM, SIZE)     # needs 44
    keys = P.Keys(1)
    d = instr([one(keys)])
    assert P.oracle_verify(bytes([2]) + d[1:17], []) == (CUSTOM, SIZE)          # 2 sigs, 16 bytes


def test_verify_outcomes():
    keys = P.Keys(2)
    assert P.oracle_verify(instr([one(keys)]), []) == (SUCCESS, 0)
    assert P.oracle_verify(instr([one(keys, b"")]), []) == (SUCCESS, 0)        # empty message
    assert P.oracle_verify(instr([one(keys, bad=True)]), []) == (CUSTOM, SIG)
    assert P.oracle_verify(instr([one(keys, k=1), one(keys, k=2, msg=b"x" * 300)]), []) == (SUCCESS, 0)
    assert P.oracle_verify(instr([one(keys), one(keys, bad=True)]), []) == (CUSTOM, SIG)


def test_fetch_rules():
    keys = P.Keys(3)
    d = bytearray(instr([one(keys)]))
    # an explicit index naming the instruction itself works like 0xFFFF
    e = bytearray(d)
    for f in (1, 3, 6):
        e[2 + 2 * f: 4 + 2 * f] = struct.pack("<H", 0)
    assert P.oracle_verify(bytes(e), [bytes(e)]) == (SUCCESS, 0)
    # an index past the txn's instructions: DATA_OFFSET (:93-94)
    for f in (1, 3, 6):
        e = bytearray(d); e[2 + 2 * f: 4 + 2 * f] = struct.pack("<H", 1)
        assert P.oracle_verify(bytes(e), [bytes(e)]) == (CUSTOM, OFFSET), f
    # a span past the data: SIGNATURE (:102-103), for each of the three spans
    for f, val in ((0, len(d) - 63), (2, len(d) - 31), (4, len(d) - 4)):
        e = bytearray(d); e[2 + 2 * f: 4 + 2 * f] = struct.pack("<H", val)
        assert P.oracle_verify(bytes(e), []) == (CUSTOM, SIG), f
    # message size 0 at the very end of the data is in range
    e = bytearray(d); e[10:12] = struct.pack("<H", len(d)); e[12:14] = struct.pack("<H", 0)
    assert P.oracle_verify(bytes(e), [])[1] in (0, SIG)


def test_first_failure_in_order_decides():
    keys = P.Keys(4)
    # record 0 fails verify, record 1 names a missing instruction: SIGNATURE
    d = bytearray(instr([one(keys, bad=True), one(keys)]))
    d[2 + 14 + 2: 2 + 14 + 4] = struct.pack("<H", 9)
    assert P.oracle_verify(bytes(d), []) == (CUSTOM, SIG)
    # record 0 names a missing instruction, record 1 fails verify: DATA_OFFSET
    d = bytearray(instr([one(keys), one(keys, bad=True)]))
    d[2 + 2: 2 + 4] = struct.pack("<H", 9)
    assert P.oracle_verify(bytes(d), []) == (CUSTOM, OFFSET)
    # within a record the signature span is checked before the pubkey span
    d = bytearray(instr([one(keys)]))
    d[2:4] = struct.pack("<H", 0xFFF0)             # sig span out of range -> SIGNATURE
    d[6:8] = struct.pack("<H", 5)                   # pubkey names a missing instruction
    assert P.oracle_verify(bytes(d), []) == (CUSTOM, SIG)


def test_cross_instruction_and_bulk_form():
    keys = P.Keys(5)
    rng = np.random.default_rng(5)
    datas, own = P.cross_instruction(keys, rng, 1)
    assert P.oracle_verify(datas[own], datas) == (SUCCESS, 0)
    assert P.oracle_verify(datas[own], datas[:1] + [b""]) == (SUCCESS, 0)   # only instruction 0 is read
    assert P.oracle_verify(datas[own], [])[1] == OFFSET
    pool, desc, tab = P.random_block(6, 300, keys)
    err, ce = P.oracle_many(pool, desc, tab)
    for j in range(desc.size):
        d = desc[j]
        instrs = [pool[t["data_off"]:t["data_off"] + t["data_sz"]].tobytes()
                  for t in tab[d["instr_base"]:d["instr_base"] + d["instr_cnt"]]]
        assert (err[j], ce[j]) == P.oracle_verify(pool[d["data_off"]:d["data_off"] + d["data_sz"]].tobytes(), instrs)
    classes = set(ce.tolist())
    assert classes == {0, SIG, OFFSET, SIZE}, classes
    assert (err == np.where(ce == 0, 0, -26)).all()
