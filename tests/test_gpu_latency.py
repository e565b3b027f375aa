"""GPU: the small-batch latency path (k_verify_lat, one workgroup of three
waves per signature) against the bulk kernels and the oracle.

Calls of at most fd_ed25519_hip_set_small_batch records (default 32, here
raised to 256) whose count is known on the host take k_verify_lat; the
drop-in entry points' single calls and the 4-record corpus KAT in the other
files already do.  Here the same records go through both paths and must give
the same codes as each other and as the oracle: mixed validity (C2
mutations), messages of 0..1232 bytes, both error modes, the full-length
(k, 1) switch, fixed-size messages, the racing copies and a bitmap."""
import numpy as np
import pytest

import oracle_lib as O
from fdgen import c2_mutate

pytestmark = pytest.mark.gpu

from firedancer_amd import ERRMODE_AVX512, ERRMODE_REF  # noqa: E402

LAT_DEFAULT = 32


@pytest.fixture
def lat(verifier):
    """the session verifier with every call of up to 256 records on k_verify_lat"""
    verifier.set_small_batch(256)
    yield verifier
    verifier.set_small_batch(LAT_DEFAULT)


def _signed_set(n, seed, max_msg=1232):
    rng = np.random.default_rng(seed)
    prvs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msz = rng.integers(0, max_msg + 1, n).astype(np.uint32)
    msz[rng.random(n) < 0.2] = 0
    moff = np.concatenate([[0], np.cumsum(msz)[:-1]]).astype(np.uint32)
    pool = rng.integers(0, 256, int(msz.sum()) + 1, dtype=np.uint8)
    pubs, sigs = O.sign_many(prvs, pool, moff, msz)
    c2_mutate(sigs, pubs, rng)
    return sigs, pubs, pool, moff, msz


def _sliced(verifier, sigs, pubs, pool, moff, msz, step):
    codes, bits = [], []
    for lo in range(0, sigs.shape[0], step):
        c, b = verifier.verify_host(sigs[lo:lo + step], pubs[lo:lo + step], pool, moff[lo:lo + step],
                                    msz[lo:lo + step])
        codes.append(c)
        bits.append(np.unpackbits(b.view(np.uint8), bitorder="little")[:c.size])
    return np.concatenate(codes), np.concatenate(bits).astype(bool)


def test_latency_path_equals_bulk_and_oracle(lat):
    verifier = lat
    sigs, pubs, pool, moff, msz = _signed_set(3000, 0x1a7)
    exp = O.verify_many(sigs, pubs, pool, moff, msz, O.ERRMODE_AVX512)
    try:
        verifier.set_small_batch(0)                              # every call through prep + DSM
        bulk, _ = verifier.verify_host(sigs, pubs, pool, moff, msz)
        verifier.set_small_batch(256)
        lat, bits = _sliced(verifier, sigs, pubs, pool, moff, msz, 200)   # every slice through k_verify_lat
    finally:
        verifier.set_small_batch(256)
    assert np.array_equal(bulk, exp)
    bad = np.nonzero(lat != exp)[0]
    assert bad.size == 0, [(int(i), int(lat[i]), int(exp[i]), int(msz[i])) for i in bad[:10]]
    assert np.array_equal(bits, lat == 0)
    assert len(set(exp.tolist())) == 4                           # every code reached


@pytest.mark.parametrize("mode", [ERRMODE_AVX512, ERRMODE_REF])
@pytest.mark.parametrize("halfsize", [1, 0])
def test_latency_path_modes(lat, mode, halfsize):
    verifier = lat
    sigs, pubs, pool, moff, msz = _signed_set(512, 0x2b8 + 7 * halfsize, max_msg=300)
    exp = O.verify_many(sigs, pubs, pool, moff, msz, mode)
    verifier.set_errmode(mode)
    verifier.set_halfsize(halfsize)
    try:
        lat, _ = _sliced(verifier, sigs, pubs, pool, moff, msz, 256)
    finally:
        verifier.set_errmode(ERRMODE_AVX512)
        verifier.set_halfsize(1)
    assert np.array_equal(lat, exp)


def test_latency_path_fixed_messages(lat):
    verifier = lat
    """verify_fixed_dev (32-byte shred-root-like messages) on the latency path."""
    import torch
    rng = np.random.default_rng(0x3c9)
    n = 200
    prvs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, n * 32 + 16, dtype=np.uint8)
    moff = (np.arange(n) * 32).astype(np.uint32)
    msz = np.full(n, 32, np.uint32)
    pubs, sigs = O.sign_many(prvs, msgs, moff, msz)
    c2_mutate(sigs, pubs, rng)
    exp = O.verify_many(sigs, pubs, msgs, moff, msz, O.ERRMODE_AVX512)
    dev = "cuda:0"
    d_sigs = torch.from_numpy(sigs.copy()).to(dev)
    d_pubs = torch.from_numpy(pubs.copy()).to(dev)
    d_msgs = torch.from_numpy(msgs.copy()).to(dev)
    codes = torch.zeros(n, dtype=torch.int8, device=dev)
    bitmap = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    verifier.verify_fixed_dev(n, d_sigs, d_pubs, d_msgs, 32, codes, bitmap)
    torch.cuda.synchronize()
    got = codes.cpu().numpy()
    assert np.array_equal(got, exp)
    bits = np.unpackbits(bitmap.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
    assert np.array_equal(bits, got == 0)


def test_latency_path_racing_copies(lat):
    verifier = lat
    """Calls of up to 32 records run one copy of each signature per XCD and
    keep the first finisher's verdict (k_verify_lat copies): slices of 1, 5,
    16 and 32 records of a mixed batch, vs the oracle."""
    sigs, pubs, pool, moff, msz = _signed_set(160, 0x4da, max_msg=400)
    exp = O.verify_many(sigs, pubs, pool, moff, msz, O.ERRMODE_AVX512)
    got = []
    lo = 0
    for step in (1, 5, 16, 32, 1, 16, 32, 5, 16, 32, 4):
        c, b = verifier.verify_host(sigs[lo:lo + step], pubs[lo:lo + step], pool, moff[lo:lo + step],
                                    msz[lo:lo + step])
        bits = np.unpackbits(b.view(np.uint8), bitorder="little")[:c.size].astype(bool)
        assert np.array_equal(bits, c == 0)
        got.append(c)
        lo += step
    got = np.concatenate(got)
    assert lo == 160 and np.array_equal(got, exp)
    for _ in range(20):                                          # repeated single calls: same verdict every time
        c, _b = verifier.verify_host(sigs[7:8], pubs[7:8], pool, moff[7:8], msz[7:8])
        assert c[0] == exp[7]


def test_default_small_batch_limit(verifier):
    """By default only calls of up to 32 records take k_verify_lat; calls of
    1..9, 31..34 records give the oracle's codes either way."""
    steps = list(range(1, 10)) + [31, 32, 33, 34]
    sigs, pubs, pool, moff, msz = _signed_set(sum(steps), 0x5eb, max_msg=200)
    exp = O.verify_many(sigs, pubs, pool, moff, msz, O.ERRMODE_AVX512)
    got, lo = [], 0
    for step in steps:
        c, _b = verifier.verify_host(sigs[lo:lo + step], pubs[lo:lo + step], pool, moff[lo:lo + step],
                                     msz[lo:lo + step])
        got.append(c)
        lo += step
    assert lo == sum(steps) and np.array_equal(np.concatenate(got), exp)
