"""The 9-limb field representation's no-overflow argument (CPU only).

tools/fe29_bounds.py mirrors every formula of firedancer_amd/csrc/
fd_ed25519_dev.h (group law, decode, table entries) with worst-case per-limb
bounds and asserts that no 64-bit column accumulator and no 32-bit limb can
overflow, and that every point coordinate stays within the tight bound the
next operation assumes.  Also checks the 2p constant and the field constants
the device code hard-codes."""
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import fe29_bounds as B  # noqa: E402

P = 2**255 - 19


def test_bounds_hold():
    assert B.check()


def test_norm_needed_where_used():
    """Dropping the normalisation of F in the doubling must be caught."""
    T = B.TIGHT
    S = B.add(T, T)
    A, Bq, C, S = B.sq(T), B.sq(T), B.sq(T), B.sq(S)
    F = B.add(B.add(C, C), B.sub(A, Bq))
    E = B.sub(B.add(A, Bq), S)
    try:
        B.mul(E, F)
    except AssertionError:
        return
    raise AssertionError("unnormalised doubling did not overflow in the tracer")


def _limbs_to_int(v):
    return sum(int(x) << (29 * i) for i, x in enumerate(v))


def test_device_constants():
    src = open(os.path.join(REPO, "firedancer_amd", "csrc", "fd_ed25519_dev.h")).read()

    def const(name):
        m = re.search(r"DEV void %s\( fe & r \)\s*\{ fe_set\( r, ([^)]*)\)" % name, src)
        return _limbs_to_int([int(x.strip().rstrip("u"), 16) for x in m.group(1).split(",")])
    d = (-121665 * pow(121666, P - 2, P)) % P
    assert const("fe_d") == d
    assert const("fe_d2") == 2 * d % P
    assert pow(const("fe_sqrtm1"), 2, P) == P - 1
    assert const("fe_inv2") * 2 % P == 1
    # 2p constant in fe_sub
    m = re.search(r"DEV void fe_sub\(.*?\n\}", src, re.S).group(0)
    c = [int(x, 16) for x in re.findall(r"\+ 0x([0-9a-f]+)u", m)]
    assert _limbs_to_int([c[0]] + [c[1]] * 7 + [c[2]]) == 2 * P


def test_pack_layout_round_trip():
    """fe_pack / fe_unpack's bit layout (8 words per element, one 30-bit limb):
    fields tile [0, 256) exactly and a pack/unpack round trip is the identity
    for limbs at their maximum widths."""
    import random
    rng = random.Random(5)
    for w30 in (0, 1):
        spans = [(B.pack_offset(w30, j), B.pack_width(w30, j)) for j in range(9)]
        pos = 0
        for o, w in spans:
            assert o == pos
            pos += w
        assert pos == 256
        cases = [[2**w - 1 for _, w in spans]] + [[rng.randrange(2**w) for _, w in spans] for _ in range(200)]
        for limbs in cases:
            x = sum(v << o for v, (o, _) in zip(limbs, spans))
            words = [(x >> (32 * k)) & 0xffffffff for k in range(8)]
            y = sum(wd << (32 * k) for k, wd in enumerate(words))
            out = [(y >> o) & (2**w - 1) for o, w in spans]
            assert out == limbs
