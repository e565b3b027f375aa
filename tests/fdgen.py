"""Test-side synthetic workload helpers: the repo's C2 mutation model plus the
message-size mix and the ten extra mutation classes that the reference-parity
tests (tests/test_gpu_ref_scale.py) and the reference-generated at-scale
fixture (tests/golden/gen_ref_scale.py) share."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd.workload import (c2_mutate, L_INT, P_INT, SMALL_ORDER_ENCODINGS,  # noqa: E402,F401
                                     KIND_VALID)

N_EXTRA = 10          # extra mutation classes, numbered 1..10 after the C2 kinds in a fixture's `extra`


def msg_sizes(rng, n, hi=1232):
    """Message sizes: 60% 0..128, 30% 128..512, 10% 512..min(hi,1232) bytes,
    5% empty; hi > 1232 adds 0.5% long messages of 1233..16383 bytes (11..129
    SHA-512 blocks with R||A)."""
    r = rng.random(n)
    msz = np.where(r < 0.6, rng.integers(0, 129, n), np.where(r < 0.9, rng.integers(128, 513, n),
                                                              rng.integers(512, min(hi, 1232) + 1, n)))
    msz[rng.random(n) < 0.05] = 0
    if hi > 1232:
        big = rng.random(n) < 0.005
        msz[big] = rng.integers(1233, 16384, int(big.sum()))
    return msz.astype(np.uint32)


def le32(x):
    return np.frombuffer(int(x).to_bytes(32, "little"), np.uint8)


def extra_mutations(rng, sigs, pubs, pool, moff, msz, valid):
    """Ten mutation classes on disjoint subsets of the still-valid records, in
    place; returns the class index lists:
      0 random R            1 random A            2 random S (mostly >= L)
      3 S in {0, L-1, L, 2^256-1}                 4 message bit flip
      5 message truncated by 1..8 bytes           6 another record's key
      7 another record's signature                8 x = 0 encodings with the sign bit set
      9 sign-bit flip of R or A"""
    idx = rng.permutation(np.nonzero(valid)[0])
    k = idx.size // 40                                  # 2.5% of the valid records per class
    cls = [idx[i * k:(i + 1) * k] for i in range(N_EXTRA)]
    n = sigs.shape[0]
    sigs[cls[0], :32] = rng.integers(0, 256, (k, 32), dtype=np.uint8)
    pubs[cls[1]] = rng.integers(0, 256, (k, 32), dtype=np.uint8)
    sigs[cls[2], 32:] = rng.integers(0, 256, (k, 32), dtype=np.uint8)
    edge_s = np.stack([le32(0), le32(L_INT - 1), le32(L_INT), le32(2 ** 256 - 1)])
    sigs[cls[3], 32:] = edge_s[rng.integers(0, 4, k)]
    for i in cls[4]:
        if msz[i]:
            b = int(rng.integers(0, 8 * int(msz[i])))
            pool[int(moff[i]) + (b >> 3)] ^= np.uint8(1 << (b & 7))
    msz[cls[5]] = np.maximum(msz[cls[5]].astype(np.int64) - rng.integers(1, 9, k), 0).astype(np.uint32)
    other = rng.integers(0, n, k)
    pubs[cls[6]] = pubs[other]
    other = rng.integers(0, n, k)
    sigs[cls[7]] = sigs[other]
    x0 = np.zeros((2, 32), np.uint8)                    # y = 1 and y = p-1 (x = 0) with the sign bit set
    x0[0, 0] = 1
    x0[0, 31] = 0x80
    x0[1] = le32(2 ** 255 - 20)
    x0[1, 31] |= 0x80
    half = k // 2
    sigs[cls[8][:half], :32] = x0[rng.integers(0, 2, half)]
    pubs[cls[8][half:]] = x0[rng.integers(0, 2, k - half)]
    sigs[cls[9][:half], 31] ^= 0x80
    pubs[cls[9][half:], 31] ^= 0x80
    return cls
