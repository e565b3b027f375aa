"""SHA-512 pinned by the reference's own CAVP vectors
(src/ballet/sha512/cavp/SHA512{Short,Long}Msg.rsp, extracted by
tests/golden/gen_cavp.py: 129 short messages of 0..128 bytes, 128 long ones of
up to 6.4 KB).

CPU: the oracle's SHA-512 (oracle/fd_ed25519_oracle.c) and hashlib on every
vector.  GPU: the device hash core k_verify_prep uses (sha512_prefixed, via
the fd_ed25519_hip_test_sha512 hook), every vector in one launch, bit-exact.
"""
import hashlib
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def cavp():
    d = np.load(os.path.join(HERE, "golden", "sha512_cavp.npz"))
    return {k: d[k] for k in d.files}


def test_fixture_shape(cavp):
    assert cavp["off"].size == 257 and (cavp["src"] == 0).sum() == 129
    assert cavp["len"].max() > 6000 and cavp["len"].min() == 0


def test_oracle_and_hashlib_match_cavp(cavp):
    import oracle_lib as O
    pool = cavp["pool"].tobytes()
    for o, n, md in zip(cavp["off"], cavp["len"], cavp["md"]):
        m = pool[o:o + n]
        assert hashlib.sha512(m).digest() == md.tobytes()
        assert O.sha512(m) == md.tobytes()


@pytest.mark.gpu
def test_device_sha512_matches_cavp(verifier, cavp):
    import torch
    dev = torch.device("cuda", 0)
    n = cavp["off"].size
    pool = torch.from_numpy(cavp["pool"]).to(dev)
    off = torch.from_numpy(cavp["off"].view(np.int32)).to(dev)
    ln = torch.from_numpy(cavp["len"].view(np.int32)).to(dev)
    out = torch.zeros((2 * n, 64), dtype=torch.uint8, device=dev)
    verifier.test_sha512(n, pool, off, ln, out)
    got = out.cpu().numpy()
    for path, g in (("per-lane", got[:n]), ("cooperative LDS", got[n:])):
        bad = np.nonzero((g != cavp["md"]).any(axis=1))[0]
        assert bad.size == 0, (path, [(int(i), int(cavp["len"][i])) for i in bad[:10]])


@pytest.mark.gpu
def test_device_sha512_unaligned_and_block_edges(verifier):
    """Every length 0..300 (all padding cases: message end at each byte of a
    128-B block, the 0x80 byte and the 16-B length straddling blocks) at all
    sixteen byte offsets mod 16 (through the 16-B pieces of the cooperative
    path), against hashlib; the pool is readable
    only 16 bytes past the last message."""
    import torch
    rng = np.random.default_rng(3)
    lens = np.repeat(np.arange(301, dtype=np.uint32), 16)
    align = np.tile(np.arange(16, dtype=np.uint32), 301)
    offs, pos = [], 0
    for n, a in zip(lens, align):
        pos = (pos + 15) // 16 * 16 + int(a)
        offs.append(pos)
        pos += int(n)
    raw = rng.integers(0, 256, pos + 16, dtype=np.uint8)
    dev = torch.device("cuda", 0)
    out = torch.zeros((2 * lens.size, 64), dtype=torch.uint8, device=dev)
    verifier.test_sha512(lens.size, torch.from_numpy(raw).to(dev),
                         torch.from_numpy(np.array(offs, np.uint32).view(np.int32)).to(dev),
                         torch.from_numpy(lens.view(np.int32)).to(dev), out)
    got = out.cpu().numpy()
    m = lens.size
    for i, (o, n) in enumerate(zip(offs, lens)):
        d = hashlib.sha512(raw[o:o + n].tobytes()).digest()
        assert got[i].tobytes() == d, ("per-lane", i, n, o % 16)
        assert got[m + i].tobytes() == d, ("cooperative LDS", i, n, o % 16)


@pytest.mark.gpu
def test_device_sha512_shared_message_runs(verifier):
    """Adjacent records sharing a message (the cooperative path loads it once
    per run and the rest of the run reads the leader's LDS copy): runs inside
    a wave and across wave boundaries, the same start with different sizes
    and the same size at different starts (neither may be merged), empty
    messages, against hashlib for both device hash paths."""
    import torch
    rng = np.random.default_rng(8)
    raw = rng.integers(0, 256, 20000, dtype=np.uint8)
    offs, lens = [], []

    def run(o, n, k):
        offs.extend([o] * k); lens.extend([n] * k)
    run(5, 200, 5); run(5, 199, 1); run(5, 200, 3); run(900, 0, 4); run(901, 0, 1)
    run(1000, 1231, 70)                       # crosses the first wave boundary (lane 63 -> 64)
    run(3000, 63, 1); run(3063, 63, 1); run(3000, 63, 2)
    for _ in range(200):                      # random runs of 1..20 over 40 distinct windows
        o = int(rng.integers(0, 40)) * 400 + int(rng.integers(0, 16)); n = int(rng.integers(0, 390))
        run(o, n, int(rng.integers(1, 21)))
    offs, lens = np.array(offs, np.uint32), np.array(lens, np.uint32)
    m = offs.size
    dev = torch.device("cuda", 0)
    out = torch.zeros((2 * m, 64), dtype=torch.uint8, device=dev)
    verifier.test_sha512(m, torch.from_numpy(raw).to(dev), torch.from_numpy(offs.view(np.int32)).to(dev),
                         torch.from_numpy(lens.view(np.int32)).to(dev), out)
    got = out.cpu().numpy()
    for i, (o, n) in enumerate(zip(offs, lens)):
        d = hashlib.sha512(raw[o:o + n].tobytes()).digest()
        assert got[i].tobytes() == d, ("per-lane", i, int(o), int(n))
        assert got[m + i].tobytes() == d, ("cooperative LDS", i, int(o), int(n))
