"""GPU: batched SHA-512 (include/fd_sha512_hip.h) and long messages through
the verify path's hash core.

Pinned by hashlib (FIPS 180-4) and the reference's own CAVP vectors
(tests/golden/sha512_cavp.npz, extracted from
src/ballet/sha512/cavp/SHA512{Short,Long}Msg.rsp by tests/golden/gen_cavp.py).
The host batching API follows fd_sha512_batch_* (fd_sha512.h:306-341).
"""
import hashlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _pack(msgs, rng=None, align=16):
    """messages back to back (16-B aligned starts, or random byte offsets),
    plus 16 readable bytes past the last one"""
    offs, pos = [], 0
    for m in msgs:
        pos = (pos + align - 1) // align * align + (int(rng.integers(0, 16)) if rng is not None else 0)
        offs.append(pos)
        pos += len(m)
    pool = np.zeros(pos + 16, np.uint8)
    for o, m in zip(offs, msgs):
        pool[o:o + len(m)] = np.frombuffer(m, np.uint8)
    return pool, np.array(offs, np.uint32), np.array([len(m) for m in msgs], np.uint32)


def _dev_hash(verifier, msgs, rng=None):
    import torch
    from firedancer_amd.sha512 import sha512_batch_dev
    dev = torch.device("cuda", 0)
    pool, off, sz = _pack(msgs, rng)
    out = torch.zeros((max(len(msgs), 1), 64), dtype=torch.uint8, device=dev)
    sha512_batch_dev(verifier, len(msgs), torch.from_numpy(pool).to(dev), torch.from_numpy(off.view(np.int32)).to(dev),
                     torch.from_numpy(sz.view(np.int32)).to(dev), out)
    return [bytes(r) for r in out.cpu().numpy()[:len(msgs)]]


def test_batch_dev_cavp(verifier):
    d = np.load(os.path.join(HERE, "golden", "sha512_cavp.npz"))
    pool = d["pool"].tobytes()
    msgs = [pool[o:o + n] for o, n in zip(d["off"], d["len"])]
    got = _dev_hash(verifier, msgs)
    assert got == [m.tobytes() for m in d["md"]]


def test_batch_dev_mixed_sizes(verifier):
    """3000 messages of 0..40 000 bytes at random byte offsets, wave-mates of
    very different block counts (including >127 blocks: the wave's maximum
    block count is taken over all 32 bits), repeated (message, size) runs
    (the shared-window path) and empty messages."""
    rng = np.random.default_rng(512)
    msgs = []
    for _ in range(3000):
        r = rng.random()
        n = int(rng.integers(0, 300)) if r < 0.6 else int(rng.integers(300, 4000)) if r < 0.9 else \
            int(rng.integers(15_000, 40_000))
        msgs.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    msgs[100:110] = [msgs[100]] * 10
    got = _dev_hash(verifier, msgs, rng)
    for i, (m, g) in enumerate(zip(msgs, got)):
        assert g == hashlib.sha512(m).digest(), (i, len(m))


def test_hash_core_long_messages(verifier):
    """Both device hash paths of k_verify_prep / k_sign (the
    fd_ed25519_hip_test_sha512 hook) on messages around the 127/128-block
    boundary (16 175 bytes: 127 blocks) and far past it."""
    import torch
    rng = np.random.default_rng(7)
    lens = [16174, 16175, 16176, 16177, 16300, 16303, 16304, 70_001, 131_072, 5]
    msgs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    pool, off, sz = _pack(msgs, rng)
    dev = torch.device("cuda", 0)
    m = len(msgs)
    out = torch.zeros((2 * m, 64), dtype=torch.uint8, device=dev)
    verifier.test_sha512(m, torch.from_numpy(pool).to(dev), torch.from_numpy(off.view(np.int32)).to(dev),
                         torch.from_numpy(sz.view(np.int32)).to(dev), out)
    got = out.cpu().numpy()
    for i, msg in enumerate(msgs):
        d = hashlib.sha512(msg).digest()
        assert got[i].tobytes() == d, ("per-lane", lens[i])
        assert got[m + i].tobytes() == d, ("cooperative LDS", lens[i])


def test_verify_long_message(verifier):
    """A 40 000-byte message (313 SHA-512 blocks with R||A) signed by the
    oracle verifies through verify_dev and the drop-in; one flipped message
    byte gives ERR_MSG in both."""
    import torch

    import oracle_lib as O
    from firedancer_amd import ed25519 as E
    rng = np.random.default_rng(40000)
    prv = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    pub = O.public_from_private(prv)
    msg = rng.integers(0, 256, 40_000, dtype=np.uint8).tobytes()
    sig = O.sign(msg, pub, prv)
    bad = bytearray(msg); bad[33_333] ^= 1; bad = bytes(bad)
    assert O.verify(msg, sig, pub) == 0 and O.verify(bad, sig, pub) == -3
    assert E.fd_ed25519_verify(msg, sig, pub) == 0
    assert E.fd_ed25519_verify(bad, sig, pub) == -3
    dev = torch.device("cuda", 0)
    pool = np.zeros(2 * 40_016 + 16, np.uint8)
    pool[:40_000] = np.frombuffer(msg, np.uint8)
    pool[40_016:80_016] = np.frombuffer(bad, np.uint8)
    sigs = torch.from_numpy(np.frombuffer(sig * 2, np.uint8).copy()).to(dev)
    pubs = torch.from_numpy(np.frombuffer(pub * 2, np.uint8).copy()).to(dev)
    codes = torch.full((2,), 9, dtype=torch.int8, device=dev)
    verifier.verify_dev(2, sigs, pubs, torch.from_numpy(pool).to(dev),
                        torch.tensor([0, 40_016], dtype=torch.int32, device=dev),
                        torch.tensor([40_000, 40_000], dtype=torch.int32, device=dev), codes)
    assert codes.cpu().tolist() == [0, -3]


def test_host_batch_api():
    """fd_sha512_hip_batch_{init,add,fini,abort} on the drop-in's context:
    5 000 records (one automatic flush at FD_SHA512_HIP_BATCH_MAX = 4096, the
    rest at fini), empty and 20 KB messages; abort drops pending records
    without writing their hashes."""
    from firedancer_amd.sha512 import BATCH_MAX, Sha512Batch, sha512_many
    rng = np.random.default_rng(4096)
    msgs = [rng.integers(0, 256, int(rng.integers(0, 2000)) if i % 97 else 20_000, dtype=np.uint8).tobytes()
            for i in range(5000)]
    msgs[3] = b""
    assert len(msgs) > BATCH_MAX
    assert sha512_many(msgs) == [hashlib.sha512(m).digest() for m in msgs]
    b = Sha512Batch()
    h = b.add(b"abc")
    b.abort()
    assert h.raw == b"\0" * 64
    assert b.fini() == []
    h = b.add(b"abc")
    assert b.fini() == [hashlib.sha512(b"abc").digest()] and h.raw == hashlib.sha512(b"abc").digest()
