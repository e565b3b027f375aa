"""GPU parity: the HIP engine (through the C ABI) against the golden fixtures
and the CPU oracle.  Bit-exact on every verdict bit and error code.

Fixtures: tests/golden/ (reference verdicts, both backends).  Oracle: oracle/
(test infrastructure only).  Sizes: KATs and ~20K random cases are compared
case by case; the 1M config-1/config-2 batches are checked through
size-independent properties (all-valid accept, rejection class per mutation
kind, bitmap == codes) plus an oracle-checked sample.
"""
import numpy as np
import pytest

import oracle_lib as O
from fdgen import c2_mutate

pytestmark = pytest.mark.gpu

from firedancer_amd import ERRMODE_AVX512, ERRMODE_REF  # noqa: E402
from firedancer_amd import ed25519 as E  # noqa: E402
from firedancer_amd import workload as W  # noqa: E402


def _records(recs):
    sigs = np.stack([np.frombuffer(bytes.fromhex(r["sig"]), np.uint8) for r in recs])
    pubs = np.stack([np.frombuffer(bytes.fromhex(r["pub"]), np.uint8) for r in recs])
    msgs = [bytes.fromhex(r["msg"]) for r in recs]
    msz = np.array([len(m) for m in msgs], np.uint32)
    moff = np.concatenate([[0], np.cumsum(msz)[:-1]]).astype(np.uint32)
    pool = np.frombuffer(b"".join(msgs) + b"\0", np.uint8)
    return sigs, pubs, pool, moff, msz


def _bitmap_ok(codes, bitmap):
    n = codes.size
    bits = np.unpackbits(bitmap.view(np.uint8), bitorder="little")[:n]
    return np.array_equal(bits.astype(bool), codes == 0)


@pytest.mark.parametrize("name", ["wycheproof", "cctv", "malleability", "corpus"])
@pytest.mark.parametrize("mode", [ERRMODE_AVX512, ERRMODE_REF])
def test_kat_bulk(verifier, kat, name, mode):
    recs = kat[name]
    verifier.set_errmode(mode)
    try:
        codes, bitmap = verifier.verify_host(*_records(recs))
    finally:
        verifier.set_errmode(ERRMODE_AVX512)
    key = "code_avx512" if mode == ERRMODE_AVX512 else "code_ref"
    exp = np.array([r[key] for r in recs], np.int8)
    bad = np.nonzero(codes != exp)[0]
    assert bad.size == 0, [(recs[i]["tc_id"], recs[i]["comment"], int(codes[i]), int(exp[i])) for i in bad[:10]]
    assert _bitmap_ok(codes, bitmap)


def test_kat_dropin_single(kat):
    """fd_ed25519_verify (link-compatible entry) on every Wycheproof vector and a
    slice of CCTV, one GPU round trip per call."""
    for r in kat["wycheproof"] + kat["cctv"][::7]:
        got = E.fd_ed25519_verify(bytes.fromhex(r["msg"]), bytes.fromhex(r["sig"]), bytes.fromhex(r["pub"]))
        assert got == r["code_avx512"], r["tc_id"]


def test_kat_dropin_batch(kat):
    for r in kat["cctv_batch"]:
        got = E.fd_ed25519_verify_batch_single_msg(bytes.fromhex(r["msg"]), bytes.fromhex(r["sigs"]),
                                                   bytes.fromhex(r["pubs"]), r["n"])
        assert got == r["code_avx512"], (r["tc_id"], r["n"])


@pytest.mark.parametrize("mode", [ERRMODE_AVX512, ERRMODE_REF])
def test_c2_mix_fixture(verifier, c2mix, mode):
    d = c2mix
    verifier.set_errmode(mode)
    try:
        codes, bitmap = verifier.verify_host(d["sigs"], d["pubs"], d["pool"], d["msg_off"], d["msg_sz"])
    finally:
        verifier.set_errmode(ERRMODE_AVX512)
    exp = d["code_avx512"] if mode == ERRMODE_AVX512 else d["code_ref"]
    bad = np.nonzero(codes != exp)[0]
    assert bad.size == 0, [(int(i), int(d["kinds"][i]), int(codes[i]), int(exp[i])) for i in bad[:10]]
    assert _bitmap_ok(codes, bitmap)


def _random_set(n, seed, max_msg=1232):
    rng = np.random.default_rng(seed)
    prvs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msz = rng.integers(0, max_msg + 1, n).astype(np.uint32)
    msz[rng.random(n) < 0.3] = 64
    moff = np.concatenate([[0], np.cumsum(msz)[:-1]]).astype(np.uint32)
    pool = rng.integers(0, 256, int(msz.sum()) + 1, dtype=np.uint8)
    pubs, sigs = O.sign_many(prvs, pool, moff, msz)
    return rng, prvs, pubs, sigs, pool, moff, msz


def test_random_mixed_vs_oracle(verifier):
    """16K oracle-signed records, messages 0..1232 B (1..10 SHA blocks), C2 mutations."""
    rng, prvs, pubs, sigs, pool, moff, msz = _random_set(16384, 0x1234)
    c2_mutate(sigs, pubs, rng)
    codes, bitmap = verifier.verify_host(sigs, pubs, pool, moff, msz)
    exp = O.verify_many(sigs, pubs, pool, moff, msz, O.ERRMODE_AVX512)
    bad = np.nonzero(codes != exp)[0]
    assert bad.size == 0, [(int(i), int(codes[i]), int(exp[i]), int(msz[i])) for i in bad[:10]]
    assert _bitmap_ok(codes, bitmap)


def test_random_bytes_vs_oracle(verifier):
    """fuzz_ed25519_verify.c:33-48 shape: uniformly random sig/pub/msg must
    not verify; codes (both error modes) equal the oracle's.  Half the S
    halves are forced < L so decode and the equation are reached too, and a
    quarter of the keys are valid points (the A decode succeeds)."""
    rng = np.random.default_rng(0xf022)
    n = 8192
    sigs = rng.integers(0, 256, (n, 64), dtype=np.uint8)
    pubs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    sigs[: n // 2, 63] &= 0x0f                                   # S < 2^252 < L
    good = O.sign_many(rng.integers(0, 256, (n // 4, 32), dtype=np.uint8), np.zeros(17, np.uint8),
                       np.zeros(n // 4, np.uint32), np.zeros(n // 4, np.uint32))[0]
    pubs[::4] = good
    msz = rng.integers(0, 300, n).astype(np.uint32)
    moff = np.concatenate([[0], np.cumsum(msz)[:-1]]).astype(np.uint32)
    pool = rng.integers(0, 256, int(msz.sum()) + 1, dtype=np.uint8)
    for mode in (O.ERRMODE_AVX512, O.ERRMODE_REF):
        verifier.set_errmode(mode)
        codes, bitmap = verifier.verify_host(sigs, pubs, pool, moff, msz)
        exp = O.verify_many(sigs, pubs, pool, moff, msz, mode)
        assert np.array_equal(codes, exp)
        assert (codes != 0).all() and _bitmap_ok(codes, bitmap)
    verifier.set_errmode(O.ERRMODE_AVX512)
    assert len(set(codes.tolist())) >= 3


def test_chunking_and_ragged(kat):
    """n not a multiple of 64, several chunks per call, empty call."""
    from firedancer_amd import Verifier
    v = Verifier(device=0, chunk_sigs=256)
    try:
        rng, prvs, pubs, sigs, pool, moff, msz = _random_set(1000, 99, max_msg=300)
        c2_mutate(sigs, pubs, rng)
        codes, bitmap = v.verify_host(sigs, pubs, pool, moff, msz)
        assert np.array_equal(codes, O.verify_many(sigs, pubs, pool, moff, msz))
        assert _bitmap_ok(codes, bitmap)
        for n in (1, 63, 65):
            c, b = v.verify_host(sigs[:n], pubs[:n], pool, moff[:n], msz[:n])
            assert np.array_equal(c, codes[:n]) and _bitmap_ok(c, b)
        c, b = v.verify_host(sigs[:0], pubs[:0], pool, moff[:0], msz[:0])
        assert c.size == 0
    finally:
        v.close()


def test_gpu_signer_matches_oracle(verifier):
    """fd_ed25519_hip_sign_dev (keygen + sign) bit-exact vs fd_ed25519_sign semantics."""
    import torch
    rng = np.random.default_rng(5)
    n = 2048
    prvs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msz = rng.integers(0, 500, n).astype(np.uint32)
    moff = np.concatenate([[0], np.cumsum(msz)[:-1]]).astype(np.uint32)
    pool = rng.integers(0, 256, int(msz.sum()) + 16, dtype=np.uint8)
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_prv, d_pool, d_off, d_sz = t(prvs), t(pool), t(moff.view(np.int32)), t(msz.view(np.int32))
    d_pub = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    d_sig = torch.zeros((n, 64), dtype=torch.uint8, device=dev)
    verifier.sign_dev(n, d_prv, d_pool, d_off, d_sz, d_pub, d_sig)
    verifier.sync()
    pubs, sigs = O.sign_many(prvs, pool, moff, msz)
    assert np.array_equal(d_pub.cpu().numpy(), pubs)
    assert np.array_equal(d_sig.cpu().numpy(), sigs)


def test_group_reduce_batch_semantics(verifier):
    """k_group_reduce == fd_ed25519_verify_batch_single_msg on random groups."""
    import torch
    rng = np.random.default_rng(11)
    msg = rng.bytes(100)
    n = 4000
    prvs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pool = np.frombuffer(msg + b"\0" * 16, np.uint8)
    moff = np.zeros(n, np.uint32); msz = np.full(n, len(msg), np.uint32)
    pubs, sigs = O.sign_many(prvs, pool, moff, msz)
    c2_mutate(sigs, pubs, rng)
    codes, _ = verifier.verify_host(sigs, pubs, pool, moff, msz)
    first, cnt = [], []
    i = 0
    while i < n:
        c = int(rng.integers(1, 17))
        c = min(c, n - i)
        first.append(i); cnt.append(c); i += c
    first += [0, 0]; cnt += [0, 17]
    dev = torch.device("cuda:0")
    d_codes = torch.from_numpy(codes).to(dev)
    d_first = torch.from_numpy(np.array(first, np.uint32).view(np.int32)).to(dev)
    d_cnt = torch.from_numpy(np.array(cnt, np.uint8)).to(dev)
    d_out = torch.zeros(len(first), dtype=torch.int8, device=dev)
    verifier.group_reduce_dev(len(first), d_first, d_cnt, d_codes, d_out)
    verifier.sync()
    got = d_out.cpu().numpy()
    for g, (f, c) in enumerate(zip(first, cnt)):
        exp = O.verify_batch_single_msg(msg, sigs[f:f + c].tobytes() if c else b"\0" * 64,
                                        pubs[f:f + c].tobytes() if c else b"\0" * 32, c)
        assert got[g] == exp, (g, f, c)


def test_full_size_c1_c2_properties(verifier):
    """Config 1/2 size (2^20 signatures, 64-B messages) resident in HBM:
    all-valid batch accepts everywhere; after the C2 mutation every rejection
    class matches its mutation kind, the bitmap equals the codes, and an
    8K sample is bit-exact against the oracle."""
    import torch
    n = 1 << 20
    batch = W.make_batch_gpu(verifier, n, msg_sz=64, seed=0x5eed0001, mix="c1")
    codes = torch.zeros(n, dtype=torch.int8, device=batch.dev)
    bitmap = torch.zeros((n + 63) // 64, dtype=torch.int64, device=batch.dev)
    verifier.verify_dev(n, batch.sigs, batch.pubs, batch.pool, batch.msg_off, batch.msg_sz, codes, bitmap)
    verifier.sync()
    assert int((codes != 0).sum()) == 0
    assert int((bitmap != -1).sum()) == 0
    # C2 mix (host-side mutation of the same records)
    sigs = batch.sigs.cpu().numpy(); pubs = batch.pubs.cpu().numpy()
    kinds = c2_mutate(sigs, pubs, np.random.default_rng(0x5eed0002))
    batch.sigs.copy_(torch.from_numpy(sigs)); batch.pubs.copy_(torch.from_numpy(pubs))
    verifier.verify_dev(n, batch.sigs, batch.pubs, batch.pool, batch.msg_off, batch.msg_sz, codes, bitmap)
    verifier.sync()
    c = codes.cpu().numpy()
    assert _bitmap_ok(c, bitmap.cpu().numpy().view(np.uint64))
    assert np.all(c[kinds == W.KIND_VALID] == 0)
    assert np.all(c[kinds == W.KIND_S_GE_L] == -1)
    assert np.all(c[kinds == W.KIND_A_SMALL] == -2)
    assert np.all(c[kinds == W.KIND_R_SMALL] == -1)
    assert np.all(c[kinds == W.KIND_SIGFLIP] != 0)
    assert np.all(c[kinds == W.KIND_PUBFLIP] != 0)
    acc = (c == 0).mean()
    assert 0.77 < acc < 0.81
    idx = np.random.default_rng(3).choice(n, 8192, replace=False)
    pool = batch.pool.cpu().numpy()
    moff = batch.msg_off.cpu().numpy().view(np.uint32); msz = batch.msg_sz.cpu().numpy().view(np.uint32)
    exp = O.verify_many(sigs[idx], pubs[idx], pool, moff[idx], msz[idx])
    assert np.array_equal(c[idx], exp)


def test_verify_host_large(verifier):
    """verify_host (host buffers, staging in HBM) on 2^18+1000 records: codes
    and bitmap equal verify_dev on the same records, and records whose
    messages are shared with other records verify as the oracle says."""
    import torch
    n = (1 << 18) + 1000
    b = W.make_batch_gpu(verifier, n, msg_sz=64, seed=0x40a7, mix="c2")
    ref = torch.zeros(n, dtype=torch.int8, device="cuda:0")
    verifier.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, ref)
    verifier.sync()
    sigs = b.sigs.cpu().numpy(); pubs = b.pubs.cpu().numpy(); pool = b.pool.cpu().numpy()
    moff = b.msg_off.cpu().numpy().view(np.uint32).copy(); msz = b.msg_sz.cpu().numpy().view(np.uint32)
    codes, bitmap = verifier.verify_host(sigs, pubs, pool, moff, msz)
    assert np.array_equal(codes, ref.cpu().numpy())
    assert _bitmap_ok(codes, bitmap)
    # second-piece records pointing at first-piece messages (pool prefix already copied)
    moff2 = moff.copy(); moff2[-5000:] = moff[:5000]
    exp = O.verify_many(sigs[-5000:], pubs[-5000:], pool, moff2[-5000:], msz[-5000:])
    codes2, _ = verifier.verify_host(sigs, pubs, pool, moff2, msz)
    assert np.array_equal(codes2[-5000:], exp)
    assert np.array_equal(codes2[:-5000], codes[:-5000])


def test_dev_count_ordered_vs_oracle():
    """The device-count path hashes in SHA-512 block-count order (k_msg_order).
    Messages 0..2600 B (1..21 blocks; keys clamp at 15) with C2 mutations,
    several 256-record chunks, device-side counts ending mid-chunk, on a chunk
    boundary and at zero: codes equal the oracle's record by record, codes
    past the count are untouched."""
    import torch
    from firedancer_amd import Verifier
    rng, prvs, pubs, sigs, pool, moff, msz = _random_set(1500, 0x0bd, max_msg=2600)
    c2_mutate(sigs, pubs, rng)
    exp = O.verify_many(sigs, pubs, pool, moff, msz)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_sigs, d_pubs, d_pool = t(sigs.reshape(-1)), t(pubs.reshape(-1)), t(pool)
    d_moff, d_msz = t(moff.view(np.int32)), t(msz.view(np.int32))
    n = sigs.shape[0]
    v = Verifier(device=0, chunk_sigs=256)
    try:
        for cnt in (n, 1000, 768, 77, 0):
            d_n = torch.tensor([cnt], dtype=torch.int32, device=dev)
            codes = torch.full((n,), 5, dtype=torch.int8, device=dev)
            v.verify_dev_count(n, d_n, d_sigs, d_pubs, d_pool, d_moff, d_msz, codes)
            v.sync()
            c = codes.cpu().numpy()
            bad = np.nonzero(c[:cnt] != exp[:cnt])[0]
            assert bad.size == 0, (cnt, [(int(i), int(c[i]), int(exp[i]), int(msz[i])) for i in bad[:10]])
            assert (c[cnt:] == 5).all(), cnt
    finally:
        v.close()
