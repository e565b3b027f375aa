"""GPU: the half-size scalar reduction inside k_verify_dsm (sc_halfsize,
firedancer_amd/csrc/fd_ed25519_dev.h) and the full-length switch.

The verdict equation [k2*S mod L]B - [k1]A - [k2]R == O equals the
reference's [S]B - [k]A == R (fd_ed25519_user.c:216-226) exactly when
k1 == k*k2 (mod 8L), k2 is odd and 0 < k2 < L.  These tests check those
invariants on crafted scalars (zero, tiny, 2^128 boundaries, L-1, scalars
whose first quotient overflows 32 bits and take the (k, 1) fallback) and on
random ones, compare the device result with the Python model
(tools/halfsize_model.py) bit for bit, and run the golden KATs with the
full-length pair (k, 1) forced for every signature."""
import os
import sys

import numpy as np
import pytest

import oracle_lib as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import halfsize_model as HM  # noqa: E402

pytestmark = pytest.mark.gpu

L = HM.L
M = HM.M


def _words(x):
    return [(x >> (32 * i)) & 0xffffffff for i in range(8)]


def _int(ws):
    return sum(int(w) << (32 * i) for i, w in enumerate(ws))


def _crafted():
    ks = [0, 1, 2, 3, 7, 8, 2**64, 2**127 - 1, 2**127, 2**128 - 1, 2**128, 2**128 + 1, 2**129 + 1,
          2**200, 2**252, L - 1, L - 2, (L - 1) // 2, M // 2**31, M // 2**32, M // (2**32 + 1),
          M // 2**33, M // 2**40, M // 3, M // 5 + 7]
    rng = np.random.default_rng(5)
    for e in range(128, 253, 4):            # one per magnitude: quotient sizes across the range
        ks.append(int(rng.integers(1, 2**62)) << (e - 62) | 1)
    return [k % L for k in ks]


def test_halfsize_invariants_and_model(verifier):
    import torch
    rng = np.random.default_rng(0x4a1f)
    ks = _crafted() + [int.from_bytes(rng.bytes(32), "little") % L for _ in range(20000)]
    n = len(ks)
    kw = np.array([_words(k) for k in ks], dtype=np.uint32)
    d_k = torch.from_numpy(kw.view(np.int32)).to("cuda:0")
    d_out = torch.zeros((n, 18), dtype=torch.int32, device="cuda:0")
    verifier.test_halfsize(n, d_k, d_out)
    verifier.sync()
    out = d_out.cpu().numpy().view(np.uint32)
    fallbacks = 0
    for i, k in enumerate(ks):
        k1 = _int(out[i, 0:8])
        k2 = _int(out[i, 8:16])
        neg, bits = int(out[i, 16]), int(out[i, 17])
        assert neg in (0, 0xffffffff)
        k1s = -k1 if neg else k1
        assert (k1s - k * k2) % M == 0, (i, k)
        assert k2 % 2 == 1 and 0 < k2 < 2**160 and k2 < L, (i, k)
        assert bits == max(k1.bit_length(), k2.bit_length()), (i, k)
        assert bits <= 253
        r, t, b, _ = HM.halfsize(k)
        assert (k1s, k2, bits) == (r, t, b), (i, k)
        if k2 == 1 and k.bit_length() > 128:
            fallbacks += 1
        if i >= len(ks) - 20000:
            assert bits <= 150, (i, k)          # random k: half size
    assert fallbacks >= 1                      # the crafted set reaches the (k, 1) path


@pytest.mark.parametrize("name", ["wycheproof", "cctv", "malleability", "corpus"])
def test_full_length_mode_kats(verifier, kat, name):
    """The golden KATs with every signature forced onto (k, 1), and on the
    default half-size path: both equal the reference's codes."""
    recs = kat[name]
    sigs = np.stack([np.frombuffer(bytes.fromhex(r["sig"]), np.uint8) for r in recs])
    pubs = np.stack([np.frombuffer(bytes.fromhex(r["pub"]), np.uint8) for r in recs])
    msgs = [bytes.fromhex(r["msg"]) for r in recs]
    msz = np.array([len(m) for m in msgs], np.uint32)
    moff = np.concatenate([[0], np.cumsum(msz)[:-1]]).astype(np.uint32)
    pool = np.frombuffer(b"".join(msgs) + b"\0", np.uint8)
    exp = np.array([r["code_avx512"] for r in recs], np.int8)
    try:
        for hs in (0, 1):
            verifier.set_halfsize(hs)
            codes, _ = verifier.verify_host(sigs, pubs, pool, moff, msz)
            bad = np.nonzero(codes != exp)[0]
            assert bad.size == 0, (hs, [(recs[i]["tc_id"], int(codes[i]), int(exp[i])) for i in bad[:10]])
    finally:
        verifier.set_halfsize(1)


def test_full_length_mode_random(verifier):
    """C2-mutated random records through both modes against the oracle."""
    import torch
    from fdgen import c2_mutate
    rng = np.random.default_rng(77)
    n = 4096
    msz = rng.integers(0, 300, n).astype(np.uint32)
    moff = np.concatenate([[0], np.cumsum(msz)[:-1]]).astype(np.uint32)
    pool = rng.integers(0, 256, int(msz.sum()) + 16, dtype=np.uint8)
    prvs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pubs, sigs = O.sign_many(prvs, pool, moff, msz)
    c2_mutate(sigs, pubs, rng)
    exp = O.verify_many(sigs, pubs, pool, moff, msz)
    dev = "cuda:0"
    args = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (sigs, pubs, pool, moff.view(np.int32),
                                                                          msz.view(np.int32))]
    try:
        for hs in (0, 1):
            verifier.set_halfsize(hs)
            codes = torch.full((n,), 9, dtype=torch.int8, device=dev)
            verifier.verify_dev(n, *args, codes)
            verifier.sync()
            assert np.array_equal(codes.cpu().numpy(), exp), hs
    finally:
        verifier.set_halfsize(1)
