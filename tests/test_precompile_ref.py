"""CPU: the oracle's restatement of the ed25519 precompile
(oracle/fd_precompile_oracle.c) pinned to the reference's own
fd_precompile_ed25519_verify (src/flamenco/runtime/program/
fd_precompiles.c:78-222), compiled here from that file where it lies and
driven through a minimal instruction context (oracle/ref_precompile_drv.c,
oracle/Makefile: _ref/libfdref_precompile.so).  Both the return value and
the custom error must be equal on every case.  The committed fixture
tests/golden/precompile_ref.npz holds the reference's answers
(tests/golden/gen_precompile_ref.py) so the pin holds where the reference
cannot be built."""
import os
import struct

import numpy as np
import pytest

import precompile_lib as P
from test_precompile_oracle import instr, one

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "precompile_ref.npz")
have_ref = pytest.mark.skipif(not os.path.exists(P.ref_path()), reason="oracle/_ref/libfdref_precompile.so not built")


def both(data, instrs):
    r = P.ref_verify(data, instrs)
    o = P.oracle_verify(data, instrs)
    assert r == o, (r, o, bytes(data)[:32].hex(), len(instrs))
    return r


@have_ref
def test_edge_cases_equal_reference():
    keys = P.Keys(11)
    for d in (b"\x00\x00", b"", b"\x00", b"\x01\x00", b"\x00\x00\x00", bytes(15), bytes(16), bytes([3, 0]) + bytes(39)):
        both(d, [])
    d = instr([one(keys)])
    assert both(d, []) == (0, 0)
    both(bytes([2]) + d[1:17], [])
    assert both(instr([one(keys, bad=True)]), []) == (-26, 2)
    both(instr([one(keys, b"")]), [])
    both(instr([one(keys), one(keys, bad=True)]), [])
    # every offset field over boundary values, with the txn holding 0, 1 and 2 instructions
    for f in range(7):
        for val in (0, 1, 2, 5, 15, 16, len(d) - 64, len(d) - 63, len(d) - 32, len(d) - 31, len(d) - 1, len(d),
                    0xFFFE, 0xFFFF):
            e = bytearray(d)
            e[2 + 2 * f: 4 + 2 * f] = struct.pack("<H", val % 0x10000)
            for instrs in ([], [bytes(e)], [bytes(e), d]):
                both(bytes(e), instrs)


@have_ref
def test_random_blocks_equal_reference():
    for seed in (1, 2, 3):
        pool, desc, tab = P.random_block(100 + seed, 600)
        rerr, rce = P.ref_many(pool, desc, tab)
        oerr, oce = P.oracle_many(pool, desc, tab)
        bad = np.nonzero((rerr != oerr) | (rce != oce))[0]
        assert bad.size == 0, [(int(j), int(rerr[j]), int(rce[j]), int(oerr[j]), int(oce[j])) for j in bad[:10]]
        assert set(rce.tolist()) == {0, 2, 3, 4}


@have_ref
def test_mutated_instructions_equal_reference():
    """Random byte and field mutations of valid multi-signature instructions."""
    keys = P.Keys(12)
    rng = np.random.default_rng(12)
    for _ in range(1500):
        nsig = int(rng.integers(1, 5))
        d = bytearray(P.self_contained(keys, rng, nsig))
        for _ in range(int(rng.integers(1, 4))):
            if rng.random() < 0.5:
                j = int(rng.integers(0, len(d))); d[j] = int(rng.integers(0, 256))
            else:
                i, f = int(rng.integers(0, nsig)), int(rng.integers(0, 7))
                d[2 + 14 * i + 2 * f: 4 + 14 * i + 2 * f] = struct.pack("<H", int(rng.integers(0, 0x10000)))
        other = rng.integers(0, 256, int(rng.integers(0, 400)), dtype=np.uint8).tobytes()
        both(bytes(d), [other, bytes(d)][:int(rng.integers(0, 3))])


def test_oracle_equals_reference_fixture():
    g = np.load(GOLD)
    oerr, oce = P.oracle_many(g["pool"], g["desc"].view(P.PC_DESC).reshape(-1), g["tab"].view(P.PC_INSTR).reshape(-1))
    assert np.array_equal(oerr, g["err"]) and np.array_equal(oce, g["custom_err"])
    assert set(g["custom_err"].tolist()) == {0, 2, 3, 4}
