#!/usr/bin/env python3
"""Worst-case limb-bound tracer for the 9-limb GF(2^255-19) representation in
firedancer_amd/csrc/fd_ed25519_dev.h (run by tests/test_fe_bounds.py).

Every field element is tracked as a list of 9 per-limb upper bounds.  Each
operation asserts the device code's no-overflow preconditions:
  mul/sq : every 64-bit column accumulator < 2^64, 2*a_i < 2^32 (sq)
  add    : every limb sum < 2^32
  sub    : the multiple-of-p constant dominates the subtrahend limb-wise
and returns the bound of its output.  The group-law sequences below mirror the
device formulas line by line (same operand order, same normalisation points);
if a formula changes there, it changes here, and the test re-proves it.
"""
import sys

R = 29
M29 = (1 << 29) - 1
M23 = (1 << 23) - 1
FOLD_HI = 1216          # 2^261 mod p  (limb 9 -> limb 0)
P = 2**255 - 19


def kp_limbs(k):
    """k*p (k = 2 or 4) as 9 limbs with every limb >= the tight bound."""
    top = (1 << 23) * k - k
    lim = [(1 << 29) * k - k] * 8 + [top]
    lim[0] -= 18 * k
    assert sum(l << (29 * i) for i, l in enumerate(lim)) == k * P
    return lim


P2, P4 = kp_limbs(2), kp_limbs(4)
U64 = 1 << 64


def _mulcols(a, b):
    """fe_mul / fe_sq: high columns 9..16 kept as unsplit 64-bit sums H_k;
    low column j = carry + products + 1216*lo32(H_{j+9}) + 9728*hi32(H_{j+8})."""
    H = []
    for k in range(9, 17):
        h = sum(a[i] * b[k - i] for i in range(k - 8, 9))
        assert h < U64, ("mul high column overflow", k, h.bit_length())
        H.append(h)
    out = [0] * 9
    acc = 0
    for k in range(9):
        acc = (0 if k == 0 else acc >> R) + sum(a[i] * b[k - i] for i in range(k + 1))
        if k < 8:
            acc += min(H[k], (1 << 32) - 1) * FOLD_HI
        if k > 0:
            acc += (H[k - 1] >> 32) * (FOLD_HI << 3)
        assert acc < U64, ("mul low column overflow", k, acc.bit_length())
        if k < 8:
            out[k] = min(acc, M29)
    out[8] = min(acc, M23)
    t = (acc >> 23) * 19 + out[0]
    assert t < U64
    out[0] = min(t, M29)
    out[1] = out[1] + (t >> R)
    assert out[1] < 1 << 32
    return out


def mul(a, b):
    return _mulcols(a, b)


def sq(a):
    assert all(2 * x < 1 << 32 for x in a), "sq: 2*a_i overflows"
    return _mulcols(a, a)


def add(a, b):
    r = [x + y for x, y in zip(a, b)]
    assert all(x < 1 << 32 for x in r), "add overflow"
    return r


def sub(a, b, k=2):
    c = P2 if k == 2 else P4
    assert all(ci >= bi for ci, bi in zip(c, b)), ("sub: %dp does not dominate b" % k)
    r = [x + ci for x, ci in zip(a, c)]
    assert all(x < 1 << 32 for x in r), "sub overflow"
    return r


def norm(a):
    a = list(a)
    for i in range(8):
        c = a[i] >> R
        a[i] = min(a[i], M29)
        a[i + 1] += c
    c = a[8] >> 23
    a[8] = min(a[8], M23)
    a[0] += 19 * c
    return a


def mx(a, b):          # bound of either operand after a conditional swap
    return [max(x, y) for x, y in zip(a, b)]


def le(a, b):
    return all(x <= y for x, y in zip(a, b))


# every mul/sq output: limbs <= M29 except limb 1 (+ (t >> 29) < 2^17, since
# the column-8 accumulator < 2^64 gives t < 19 * 2^41 + 2^29) and limb 8 <= M23
TIGHT = [M29, M29 + (1 << 17)] + [M29] * 6 + [M23]
WORDS = [M29] * 8 + [M23]             # fe_from_words of any 32-byte string


# ---- group law (mirrors fd_ed25519_dev.h) -------------------------------
def ge_dbl(P, needT):
    X, Y, Z = P[:3]
    S = add(X, Y)
    A, B, C, S = sq(X), sq(Y), sq(Z), sq(S)
    C2 = add(C, C)
    H = add(A, B)
    G = sub(A, B)
    F = norm(add(C2, G))
    E = sub(H, S)
    if needT:
        E = norm(E)
    out = [mul(E, F), mul(G, H), mul(F, G)]
    out.append(mul(E, H) if needT else None)
    return out


def ge_add(P, q, affine):
    """q = (YmX, YpX, T2d[, Z2]) table entries; neg swaps YmX/YpX and F/G.
    affine: True (1/2-scaled affine entry, D = Z1), False (cached, D = Z1*Z2)
    or "z1" (ge_add_cached_z1: cached form of an affine point, D = norm(2 Z1))."""
    X, Y, Z, T = P
    qa = qb = mx(q[0], q[1])
    a = sub(Y, X)
    b = add(Y, X)
    A, B, C = mul(a, qa), mul(b, qb), mul(T, q[2])
    if affine == "z1":
        D = norm(add(Z, Z))
    else:
        D = Z if affine else mul(Z, q[3])
    E = norm(sub(B, A))
    H = add(B, A)
    F = sub(D, C)
    G = add(D, C)
    Fs = Gs = mx(F, G)
    return [mul(E, Fs), mul(Gs, H), mul(F, G), mul(E, H)]


def pack_width(w30, j):
    """limb j's field width in an 8-word packed element (fe_pack_layout)"""
    return 23 if j == 8 else (30 if j == w30 else 29)


def pack_offset(w30, j):
    return 0 if j == 0 else (0 if j <= w30 else 1) + 29 * j


def check():
    pt = [TIGHT] * 4
    for needT in (False, True):
        r = ge_dbl(pt, needT)
        assert all(le(o, TIGHT) for o in r if o), "dbl output not tight"
    # A-table entries (ge_to_cached): norm(Y-X), norm(Y+X), T*2d, norm(2Z)
    entry = [norm(sub(TIGHT, TIGHT)), norm(add(TIGHT, TIGHT)), TIGHT, norm(add(TIGHT, TIGHT))]
    for affine in (False, True, "z1"):
        r = ge_add(pt, entry, affine)
        assert all(le(o, TIGHT) for o in r), "add output not tight"
    # packed table entries (fe_pack<W30>, fd_ed25519_hip.hip): Y-X, Y+X, 2Z
    # with the wide limb 0, 2d*T with the wide limb 1
    for e, w30 in zip(entry, (0, 0, 1, 0)):
        assert all(v < 2**pack_width(w30, j) for j, v in enumerate(e)), "table element does not pack"
    # decode (ge_decode): y from words
    one = [1] + [0] * 8
    y2 = sq(WORDS)
    u = sub(y2, one)
    v = add(mul(y2, TIGHT), one)
    v3 = mul(sq(v), v)
    mul(u, mul(sq(v3), v))
    mul(mul(u, v3), TIGHT)
    return True


if __name__ == "__main__":
    print("2p limbs", P2)
    print("tight   ", TIGHT)
    try:
        check()
    except AssertionError as e:
        print("BOUND VIOLATION:", e)
        sys.exit(1)
    print("all group-law and decode bounds hold")
