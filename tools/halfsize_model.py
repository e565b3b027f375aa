"""Model of the device half-size scalar reduction (sc_halfsize in
firedancer_amd/csrc/fd_ed25519_dev.h): truncated Euclid on (8L, k) with
cofactors, float quotients with exact correction, best odd-cofactor vector
among three consecutive remainders and their +-1 combinations.

Checks k1 == k*k2 (mod 8L), k2 odd and > 0, and prints the distribution of
the window count D = floor(bits/4) + 1 (digits in [-7, 8]) per lane and per
64-lane wave (in index order, and after k_verify_scalar's bucketing of short
and long lanes), and of the Euclid iteration count.

Usage: python tools/halfsize_model.py [n]"""
import collections
import math
import random
import sys

L = 2**252 + 27742317777372353535851937790883648493
M = 8 * L


def qstep(dp, dc):
    """floor of the float quotient; None when it does not fit 32 bits (the
    lane then takes the full-length scalars (k, 1): probability ~2^-30)"""
    q = math.floor(dp / dc)
    return q if q < 2**32 else None


def halfsize(k):
    rp, rc, tp, tc = M, k, 0, 1
    dp, dc = float(M), float(k)
    it = 0
    while rc >= 2**128:
        q = qstep(dp, dc)
        if q is None:
            return k, 1, k.bit_length(), it
        rn, tn = rp - q * rc, tp - q * tc
        if rn < 0:
            rn, tn = rn + rc, tn + tc
        if rn >= rc:
            rp, tp, dp = rn, tn, float(rn)
        else:
            rp, tp, rc, tc, dp, dc = rc, tc, rn, tn, dc, float(rn)
        it += 1
    q = qstep(dp, dc) if rc else None
    if q is not None and q < 2**30:
        rn, tn = rp - q * rc, tp - q * tc
        if rn < 0:
            rn, tn = rn + rc, tn + tc
    else:
        rn, tn = rp, tp
    v = [(rp, tp), (rc, tc), (rn, tn)]
    cands = list(v)
    for i, j in ((0, 1), (0, 2), (1, 2)):
        cands.append((v[i][0] + v[j][0], v[i][1] + v[j][1]))
        cands.append((v[i][0] - v[j][0], v[i][1] - v[j][1]))
    best = None
    for r, t in cands:
        if t % 2 == 0:
            continue
        b = max(abs(r).bit_length(), abs(t).bit_length())
        if best is None or b < best[0]:
            best = (b, r, t)
    b, r, t = best
    if b > 250:
        b, r, t = k.bit_length(), k, 1
    if t < 0:
        r, t = -r, -t
    assert t > 0 and t % 2 == 1 and (r - k * t) % M == 0
    return r, t, b, it


def windows(b):
    return b // 4 + 1


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64 * 2000
    rng = random.Random(7)
    ks = [rng.randrange(L) for _ in range(n)] + [0, 1, 2**128 - 1, 2**128, L - 1, 8, 2**200, 2**129 + 1]
    D, its, wd, wi = collections.Counter(), collections.Counter(), collections.Counter(), collections.Counter()
    lane_d, lane_i = [], []
    for k in ks:
        r, t, b, it = halfsize(k)
        D[windows(b)] += 1
        its[it] += 1
        lane_d.append(max(31, windows(b)))
        lane_i.append(it)
    for i in range(0, n, 64):
        wd[max(lane_d[i:i + 64])] += 1
        wi[max(lane_i[i:i + 64])] += 1
    # k_verify_scalar's bucketing: lanes with D <= 32 listed first, the rest after
    ld = lane_d[:n]
    srt = [d for d in ld if d <= 32] + [d for d in ld if d > 32]
    wb = [max(srt[i:i + 64]) for i in range(0, n, 64)]
    print("lane windows", sorted(D.items()))
    print("bucketed wave windows mean", sum(wb) / len(wb), "lane mean", sum(ld) / len(ld))
    print("wave windows", sorted(wd.items()), "mean", sum(k * v for k, v in wd.items()) / sum(wd.values()))
    print("lane iters mean", sum(lane_i) / len(lane_i), "wave iters mean", sum(k * v for k, v in wi.items()) / sum(wi.values()),
          "max", max(lane_i))


if __name__ == "__main__":
    main()
