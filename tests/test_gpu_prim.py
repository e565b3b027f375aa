"""GPU: the device primitives under k_verify_prep / k_verify_dsm, one at a
time, through the fd_ed25519_hip_test_prim hook (include/fd_ed25519_hip.h).

The reference unit-tests its field, point and scalar layers separately
(test_ed25519.c: test_fe_* :53-604, test_affine_frombytes :605,
test_affine_is_small_order :615, test_point_frombytes :718, test_sc_validate
:882, test_sc_reduce :909).  This file does the same for the device code:
  - GF(2^255-19) multiply / square (single and interleaved pairs) at every
    operand bound the group-law and decode formulas produce (recorded from
    tools/fe29_bounds.py's worst-case tracer), all-maximum limbs included,
    against Python big integers: value mod p and tight output limbs;
  - canonicalisation of arbitrary limbs (values around p, 2p, 2^255 and
    every limb at its maximum), byte decoding with non-canonical y in
    [p, 2^255), subtraction, pow22523 and inversion;
  - point decoding with the AVX-512 failure split and the small-order test,
    against the oracle's restatement (oracle_point_decode /
    oracle_point_is_small_order) on random, small-order, non-canonical and
    x = 0 encodings;
  - scalar reduction mod L and S < L on edge values.
"""
import os
import sys

import numpy as np
import pytest

import oracle_lib as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

pytestmark = pytest.mark.gpu

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
M29 = 2**29 - 1
TIGHT = [M29, 2**29 + 2**17 - 1] + [M29] * 6 + [2**23 - 1]

OPS = dict(FE_MUL=0, FE_SQ=1, FE_MUL2=2, FE_SQ2=3, FE_CANON=4, FE_FROMWORDS=5, FE_SUB=6, FE_POW22523=7,
           FE_INVERT=8, GE_DECODE=9, SC_REDUCE=10, SC_CANONICAL=11)


def val(limbs):
    return sum(int(x) << (29 * i) for i, x in enumerate(limbs))


def limbs_of(x):
    """canonical 9-limb form of 0 <= x < 2^255"""
    return [(x >> (29 * i)) & (M29 if i < 8 else 2**23 - 1) for i in range(9)]


def is_tight(limbs):
    return all(int(x) <= t for x, t in zip(limbs, TIGHT))


def is_canonical(limbs):
    return all(int(x) <= (M29 if i < 8 else 2**23 - 1) for i, x in enumerate(limbs)) and val(limbs) < P


def words_of(x, n=8):
    return [(x >> (32 * i)) & 0xffffffff for i in range(n)]


def rand_limbs(rng, bound, k):
    """k random limb vectors with limb i in [0, bound[i]]: uniform, plus the
    all-maximum, all-zero and alternating-extreme vectors"""
    b = np.array(bound, dtype=np.uint64)
    r = (rng.integers(0, 2**63, size=(k, 9), dtype=np.uint64) % (b + 1)).astype(np.uint64)
    ext = [b, np.zeros(9, np.uint64), np.where(np.arange(9) % 2 == 0, b, 0), np.where(np.arange(9) % 2 == 1, b, 0),
           np.maximum(b - 1, 0)]
    return np.vstack([np.array(ext, dtype=np.uint64), r]).astype(np.uint32)


def run(verifier, op, inp):
    import torch
    n = inp.shape[0]
    buf = np.zeros((n, 32), dtype=np.uint32)
    buf[:, :inp.shape[1]] = inp
    d_in = torch.from_numpy(buf.view(np.int32)).to("cuda:0")
    d_out = torch.zeros((n, 32), dtype=torch.int32, device="cuda:0")
    verifier.test_prim(OPS[op], n, d_in, d_out)
    verifier.sync()
    return d_out.cpu().numpy().view(np.uint32)


def proven_operand_bounds():
    """Every (a, b) operand-bound pair of a multiply and every operand bound of
    a square that the group-law and decode formulas produce, recorded by
    running tools/fe29_bounds.py's worst-case tracer (it mirrors
    fd_ed25519_dev.h formula by formula)."""
    import fe29_bounds as F
    muls, sqs = set(), set()
    m0, s0 = F.mul, F.sq

    def rec_mul(a, b):
        muls.add((tuple(a), tuple(b)))
        return m0(a, b)

    def rec_sq(a):
        sqs.add(tuple(a))
        return s0(a)

    F.mul, F.sq = rec_mul, rec_sq
    try:
        assert F.check()
    finally:
        F.mul, F.sq = m0, s0
    return sorted(muls), sorted(sqs)


def test_fe_mul_at_proven_operand_bounds(verifier):
    muls, _ = proven_operand_bounds()
    assert len(muls) >= 8
    rng = np.random.default_rng(11)
    a = np.vstack([rand_limbs(rng, ab, 600) for ab, _ in muls])
    b = np.vstack([rand_limbs(rng, bb, 600) for _, bb in muls])
    out = run(verifier, "FE_MUL", np.hstack([a, b]))
    out2 = run(verifier, "FE_MUL2", np.hstack([a, b]))
    for i in range(a.shape[0]):
        e = (val(a[i]) * val(b[i])) % P
        for o in (out[i, 0:9], out2[i, 0:9], out2[i, 9:18]):
            assert val(o) % P == e and is_tight(o), (i, list(a[i]), list(b[i]))


def test_fe_sq_at_proven_operand_bounds(verifier):
    _, sqs = proven_operand_bounds()
    rng = np.random.default_rng(12)
    a = np.vstack([rand_limbs(rng, ab, 1000) for ab in sqs])
    b = np.vstack([rand_limbs(rng, ab, 1000) for ab in sqs])
    out = run(verifier, "FE_SQ", np.hstack([a, b]))
    out2 = run(verifier, "FE_SQ2", np.hstack([a, b]))
    for i in range(a.shape[0]):
        va, vb = val(a[i]), val(b[i])
        for o, e in ((out[i, 0:9], va * va), (out2[i, 0:9], va * va), (out2[i, 9:18], vb * vb)):
            assert val(o) % P == e % P and is_tight(o), (i, list(a[i]))


def test_fe_canon_edges(verifier):
    rng = np.random.default_rng(13)
    vals = [0, 1, P - 1, P, P + 1, 2 * P - 1, 2 * P, 2 * P + 18, 2**255 - 1, 2**255, 2**255 + 18, 2**256 - 1]
    rows = [limbs_of(v % 2**255) + [0] * 0 for v in vals if v < 2**255]
    # values >= 2^255 spelled with an oversized top limb (limb 8 holds bits 232 up)
    for v in vals:
        if v >= 2**255:
            lo = [(v >> (29 * i)) & M29 for i in range(8)]
            rows.append(lo + [v >> 232])
    # every limb at the largest value fe_norm takes (< 2^32 - 8)
    rows.append([2**32 - 9] * 9)
    r = rng.integers(0, 2**32 - 8, size=(4000, 9), dtype=np.uint64)
    inp = np.vstack([np.array(rows, dtype=np.uint64), r]).astype(np.uint32)
    out = run(verifier, "FE_CANON", inp)
    for i in range(inp.shape[0]):
        assert is_canonical(out[i, :9]) and val(out[i, :9]) == val(inp[i]) % P, (i, list(inp[i]))


def test_fe_frombytes_keeps_noncanonical_y(verifier):
    """fd_f25519_frombytes (test_fe_frombytes, test_ed25519.c:53-101): bit 255
    is dropped, y in [p, 2^255) is kept as is (reduced by later arithmetic)."""
    rng = np.random.default_rng(14)
    xs = [0, 1, P - 1, P, P + 1, P + 18, 2**255 - 1, 2**255, 2**256 - 1, 2**255 + P]
    xs += [int.from_bytes(rng.bytes(32), "little") for _ in range(4000)]
    inp = np.array([words_of(x) for x in xs], dtype=np.uint32)
    out = run(verifier, "FE_FROMWORDS", inp)
    for i, x in enumerate(xs):
        assert [int(w) for w in out[i, :9]] == limbs_of(x & (2**255 - 1)), i


def test_fe_sub_pow_invert(verifier):
    """a - b, a^(2^252-3) (test_fe_pow22523, test_ed25519.c:531-604) and
    a^(p-2) (test_fe_invert :405-430) on tight inputs, canonical out."""
    rng = np.random.default_rng(15)
    a = rand_limbs(rng, TIGHT, 1500)
    b = rand_limbs(rng, TIGHT, 1500)
    special = np.array([limbs_of(v) for v in (0, 1, 2, P - 1, P - 2, 2**254, 19)], dtype=np.uint32)
    a = np.vstack([special, a])
    b = np.vstack([special[::-1], b[:a.shape[0] - special.shape[0]]])
    ab = np.hstack([a, b])
    sub = run(verifier, "FE_SUB", ab)
    pw = run(verifier, "FE_POW22523", ab)
    inv = run(verifier, "FE_INVERT", ab)
    e = 2**252 - 3
    for i in range(a.shape[0]):
        va, vb = val(a[i]) % P, val(b[i]) % P
        assert is_canonical(sub[i, :9]) and val(sub[i, :9]) == (va - vb) % P, i
        assert is_canonical(pw[i, :9]) and val(pw[i, :9]) == pow(va, e, P), i
        assert is_canonical(inv[i, :9]) and val(inv[i, :9]) == pow(va, P - 2, P), i


def _decode_cases(rng):
    encs = []
    # the 8 small-order points' encodings, canonical and with y + p where that fits
    # (fd_curve25519.h:91-98 lists them; y0/y1 from table/fd_curve25519_table_ref.c:18-27)
    y0 = val([0x0f95e826, 0x013d9614, 0x1d30d16c, 0x11dfe513, 0x0dfd5f09, 0x036982d6, 0x02c4e4cf, 0x0db10047,
              0x0005fc53])
    y1 = (P - y0) % P
    for y in (0, 1, P - 1, y0, y1):
        for sign in (0, 1):
            for yy in (y, y + P):
                if yy < 2**255:
                    encs.append(yy | (sign << 255))
    # x = 0 with the sign bit set (AVX-512 rejects in decode), and y >= p near the top
    for y in (1, P - 1, P + 1, 2**255 - 1, 2**255 - 19, P - 2):
        encs.append(y | (1 << 255))
        encs.append(y)
    # random encodings (about half are not on the curve) and GPU-free valid points
    encs += [int.from_bytes(rng.bytes(32), "little") for _ in range(3000)]
    for j in range(200):
        pub = O.public_from_private(rng.bytes(32))
        encs.append(int.from_bytes(pub, "little"))
    return encs


def test_ge_decode_and_small_order_vs_oracle(verifier):
    """fd_ed25519_point_frombytes / affine_is_small_order (test_point_frombytes
    :718-761, test_affine_is_small_order :615-670) against the oracle."""
    import ctypes
    rng = np.random.default_rng(16)
    encs = _decode_cases(rng)
    inp = np.array([words_of(x) for x in encs], dtype=np.uint32)
    out = run(verifier, "GE_DECODE", inp)
    lib = O.lib()
    seen = {0: 0, 1: 0, 2: 0}
    small = 0
    for i, x in enumerate(encs):
        buf = x.to_bytes(32, "little")
        xy = ctypes.create_string_buffer(64)
        rc = lib.oracle_point_decode(xy, buf)
        seen[rc] += 1
        flags = int(out[i, 0])
        exp_flags = {0: 0, 1: 1, 2: 2}[rc]
        assert flags == exp_flags, (i, hex(x), flags, rc)
        if rc != 1:
            gx = b"".join(int(w).to_bytes(4, "little") for w in out[i, 2:10])
            gy = b"".join(int(w).to_bytes(4, "little") for w in out[i, 10:18])
            assert gx + gy == xy.raw, (i, hex(x))
            so = lib.oracle_point_is_small_order(buf)
            assert int(out[i, 1]) == so, (i, hex(x))
            small += so
    assert seen[0] > 1000 and seen[1] > 1000 and seen[2] >= 2 and small >= 10


def test_sc_reduce_and_validate_edges(verifier):
    """fd_curve25519_scalar_reduce (test_sc_reduce :909-933) and
    scalar_validate (test_sc_validate :882-908)."""
    rng = np.random.default_rng(17)
    xs = [0, 1, L - 1, L, L + 1, 2 * L, 2**252, 2**253 - 1, 2**256 - 1, 2**512 - 1, L * (2**259 - 1),
          L * (2**259) - 1, (2**512 // L) * L, (2**512 // L) * L - 1]
    xs += [int.from_bytes(rng.bytes(64), "little") for _ in range(3000)]
    inp = np.array([words_of(x, 16) for x in xs], dtype=np.uint32)
    out = run(verifier, "SC_REDUCE", inp)
    for i, x in enumerate(xs):
        got = sum(int(w) << (32 * k) for k, w in enumerate(out[i, :8]))
        assert got == x % L, i
        assert got.to_bytes(32, "little") == O.scalar_reduce(x.to_bytes(64, "little")), i
    ss = [0, 1, L - 2, L - 1, L, L + 1, 2**253 - 1, 2**255, 2**256 - 1, L + 2**128]
    ss += [int.from_bytes(rng.bytes(32), "little") >> int(rng.integers(0, 5)) for _ in range(3000)]
    inp = np.array([words_of(s) for s in ss], dtype=np.uint32)
    out = run(verifier, "SC_CANONICAL", inp)
    for i, s in enumerate(ss):
        assert int(out[i, 0]) == (1 if s < L else 0), (i, hex(s))


def test_unknown_op_rejected(verifier):
    import torch
    d = torch.zeros((1, 32), dtype=torch.int32, device="cuda:0")
    with pytest.raises(ValueError):
        verifier.test_prim(99, 1, d, d)
