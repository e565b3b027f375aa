"""CPU: the oracle (oracle/liboracle.so) against the reference's own vectors.

Pins the restatement before it is used as the GPU checker (tests/golden/ holds
the reference's Wycheproof / CCTV / malleability / corpus vectors with the
verdicts and error codes of the reference build, both backends)."""
import hashlib
import os

import numpy as np
import pytest

import oracle_lib as O

KAT_SETS = ("wycheproof", "cctv", "malleability", "corpus")


@pytest.mark.parametrize("name", KAT_SETS)
def test_oracle_kat_codes(kat, name):
    recs = kat[name]
    assert recs
    for r in recs:
        m, s, p = bytes.fromhex(r["msg"]), bytes.fromhex(r["sig"]), bytes.fromhex(r["pub"])
        assert O.verify(m, s, p, O.ERRMODE_AVX512) == r["code_avx512"], (name, r["tc_id"])
        assert O.verify(m, s, p, O.ERRMODE_REF) == r["code_ref"], (name, r["tc_id"])
        if "ok" in r:
            assert (r["code_avx512"] == 0) == bool(r["ok"])


def test_oracle_vector_counts(kat):
    # test_ed25519_wycheproof.c:22 (133), test_ed25519_cctv.c:22 (914),
    # malleability .bin sizes 18816/96 + 19200/96
    assert len(kat["wycheproof"]) == 133
    assert len(kat["cctv"]) == 914
    assert len(kat["malleability"]) == 196 + 200
    assert sum(r["ok"] for r in kat["wycheproof"]) == 84
    assert sum(r["ok"] for r in kat["cctv"]) == 43


def test_oracle_batch_single_msg(kat):
    for r in kat["cctv_batch"]:
        m = bytes.fromhex(r["msg"])
        for mode, key in ((O.ERRMODE_AVX512, "code_avx512"), (O.ERRMODE_REF, "code_ref")):
            got = O.verify_batch_single_msg(m, bytes.fromhex(r["sigs"]), bytes.fromhex(r["pubs"]), r["n"], mode)
            assert got == r[key], (r["tc_id"], r["n"])


def test_oracle_c2_mix(c2mix):
    d = c2mix
    for mode, key in ((O.ERRMODE_AVX512, "code_avx512"), (O.ERRMODE_REF, "code_ref")):
        codes = O.verify_many(d["sigs"], d["pubs"], d["pool"], d["msg_off"], d["msg_sz"], mode)
        assert np.array_equal(codes, d[key])
    acc = (d["code_avx512"] == 0).mean()
    assert 0.74 < acc < 0.84          # ~79% accepted in the C2 mix


def test_oracle_sign_kat(kat):
    k = kat["sign_kat"][0]
    prv = bytes.fromhex(k["prv"])
    assert O.public_from_private(prv).hex() == k["pub"]
    assert O.sign(b"", bytes.fromhex(k["pub"]), prv).hex() == k["sig"]
    for c in kat["corpus"]:
        assert O.sign(bytes.fromhex(c["msg"]), bytes.fromhex(c["pub"]), bytes.fromhex(c["prv"])).hex() == c["sig"]


def test_oracle_sha512():
    rng = np.random.default_rng(7)
    for n in (0, 1, 111, 112, 127, 128, 129, 239, 240, 1000, 1232):
        b = rng.bytes(n)
        assert O.sha512(b) == hashlib.sha512(b).digest()


def test_oracle_scalar_reduce():
    L = 2**252 + 27742317777372353535851937790883648493
    rng = np.random.default_rng(8)
    for _ in range(200):
        b = rng.bytes(64)
        assert int.from_bytes(O.scalar_reduce(b), "little") == int.from_bytes(b, "little") % L
    for v in (0, L - 1, L, L + 1, 2**512 - 1, 2**253, L * (2**259)):
        b = v.to_bytes(64, "little")
        assert int.from_bytes(O.scalar_reduce(b), "little") == v % L


REF_AVX = os.path.join(O.ORACLE_DIR, "_ref", "libfdref_avx512.so")


@pytest.mark.skipif(not os.path.exists(REF_AVX), reason="reference build (oracle/_ref) absent")
def test_oracle_vs_reference_build_random():
    """Live differential check against the reference compiled from its sources."""
    import ctypes
    sys_path_golden = os.path.join(os.path.dirname(__file__), "golden")
    import sys
    sys.path.insert(0, sys_path_golden)
    from gen_golden import RefLib
    from fdgen import c2_mutate
    for path, mode in ((REF_AVX, O.ERRMODE_AVX512), (REF_AVX.replace("avx512", "ref"), O.ERRMODE_REF)):
        if "avx512" in path and not _cpu_has_avx512ifma():
            continue
        ref = RefLib(path)
        rng = np.random.default_rng(0xabc + mode)
        n = 1500
        prvs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        msz = rng.integers(0, 200, n).astype(np.uint32)
        moff = np.concatenate([[0], np.cumsum(msz)[:-1]]).astype(np.uint32)
        pool = rng.integers(0, 256, int(msz.sum()) + 1, dtype=np.uint8)
        pubs, sigs = O.sign_many(prvs, pool, moff, msz)
        c2_mutate(sigs, pubs, rng)
        got = O.verify_many(sigs, pubs, pool, moff, msz, mode)
        for i in range(n):
            m = pool[moff[i]:moff[i] + msz[i]].tobytes()
            assert got[i] == ref.verify(m, sigs[i].tobytes(), pubs[i].tobytes()), i


def _cpu_has_avx512ifma():
    try:
        return "avx512ifma" in open("/proc/cpuinfo").read()
    except OSError:
        return False
