"""GPU: stream ordering of a context's shared scratch, the bitmap's partial
last word, and full-size config 3.

- Two verifies on ONE context issued back to back on two different streams
  (no host sync between them) must both give the codes each gives alone:
  the context orders its scratch use with an event (fd_ed25519_hip.h).
- A device-count verify whose count ends inside a bitmap word leaves the
  bits at or past the count untouched (include/fd_ed25519_hip.h).
- C3 at its BASELINE size: one 32-B message x 2^22 keys, all valid, as
  fd_ed25519_verify_batch_single_msg groups of 16 (fd_ed25519_user.c:232-310):
  every signature and every group SUCCESS; a sample of groups equals the
  oracle's batch verify with one signature corrupted per group.
"""
import numpy as np
import pytest
import torch

import oracle_lib as O
from firedancer_amd import workload as W

pytestmark = pytest.mark.gpu


def test_two_streams_one_context(verifier):
    dev = torch.device("cuda", 0)
    n = 1 << 18
    a = W.make_batch_gpu(verifier, n, msg_sz=64, seed=0xa11, mix="c2")
    b = W.make_batch_gpu(verifier, n, msg_sz=100, seed=0xb22, mix="c2")
    ref_a = torch.zeros(n, dtype=torch.int8, device=dev)
    ref_b = torch.zeros(n, dtype=torch.int8, device=dev)
    verifier.verify_dev(n, a.sigs, a.pubs, a.pool, a.msg_off, a.msg_sz, ref_a)
    verifier.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, ref_b)
    torch.cuda.synchronize()
    assert not torch.equal(ref_a, ref_b)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for rep in range(3):
        ca = torch.full((n,), 9, dtype=torch.int8, device=dev)
        cb = torch.full((n,), 9, dtype=torch.int8, device=dev)
        torch.cuda.synchronize()
        verifier.verify_dev(n, a.sigs, a.pubs, a.pool, a.msg_off, a.msg_sz, ca, stream=s1.cuda_stream)
        verifier.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, cb, stream=s2.cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(ca, ref_a), rep
        assert torch.equal(cb, ref_b), rep


def test_bitmap_partial_word_untouched(verifier):
    dev = torch.device("cuda", 0)
    n = 4096
    b = W.make_batch_gpu(verifier, n, msg_sz=64, seed=0x77, mix="c2")
    ref = torch.zeros(n, dtype=torch.int8, device=dev)
    verifier.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, ref)
    r = ref.cpu().numpy()
    for cnt in (1000 + 17, 64 * 7, 1, 4095):
        d_n = torch.tensor([cnt], dtype=torch.int32, device=dev)
        codes = torch.full((n,), 9, dtype=torch.int8, device=dev)
        bm = torch.full(((n + 63) // 64,), -1, dtype=torch.int64, device=dev)      # every bit set
        verifier.verify_dev_count(n, d_n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes, bm)
        bits = np.unpackbits(bm.cpu().numpy().view(np.uint8), bitorder="little").astype(bool)
        assert np.array_equal(bits[:cnt], r[:cnt] == 0), cnt
        assert bits[cnt:].all(), (cnt, int((~bits[cnt:]).sum()))


def test_c3_full_size_groups_of_16(verifier):
    dev = torch.device("cuda", 0)
    n = 1 << 22
    b = W.make_batch_gpu(verifier, n, msg_sz=32, seed=0xc3, mix="c1", shared_msg=True)
    codes = torch.full((n,), 9, dtype=torch.int8, device=dev)
    bm = torch.zeros(n // 64, dtype=torch.int64, device=dev)
    verifier.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes, bm)
    ng = n // 16
    first = torch.arange(ng, dtype=torch.int32, device=dev) * 16
    cnt = torch.full((ng,), 16, dtype=torch.uint8, device=dev)
    g = torch.full((ng,), 9, dtype=torch.int8, device=dev)
    verifier.group_reduce_dev(ng, first, cnt, codes, g)
    assert int((codes != 0).sum()) == 0
    assert int((bm != -1).sum()) == 0
    assert int((g != 0).sum()) == 0
    # 64 sampled groups with one corrupted signature each, against the oracle's batch verify
    rng = np.random.default_rng(33)
    msg = b.pool[:32].cpu().numpy().tobytes()
    for grp in rng.choice(ng, 64, replace=False):
        s = b.sigs[16 * grp:16 * grp + 16].cpu().numpy().copy()
        p = b.pubs[16 * grp:16 * grp + 16].cpu().numpy()
        j, bit = int(rng.integers(0, 16)), int(rng.integers(0, 512))
        s[j, bit >> 3] ^= 1 << (bit & 7)
        exp = O.verify_batch_single_msg(msg, s.tobytes(), p.tobytes(), 16)
        ds = torch.from_numpy(s).to(dev)
        c16 = torch.full((16,), 9, dtype=torch.int8, device=dev)
        verifier.verify_dev(16, ds, b.pubs[16 * grp:16 * grp + 16], b.pool, b.msg_off[:16], b.msg_sz[:16], c16)
        g1 = torch.full((1,), 9, dtype=torch.int8, device=dev)
        verifier.group_reduce_dev(1, first[:1], cnt[:1], c16, g1)
        assert int(g1.item()) == exp != 0, (grp, j, bit)


def test_cu_masked_context_stream():
    """fd_ed25519_hip_ctx_set_cu_mask: a context whose stream runs on 8 CUs
    only (bulk path, 4096 C2 records, and a latency-path call of 12) gives
    the oracle's codes, and returns to every CU with an empty mask."""
    from firedancer_amd import Verifier
    from firedancer_amd.ed25519 import CTX_STREAM
    v = Verifier(device=0, chunk_sigs=1 << 14)
    try:
        assert v.set_cu_mask([0, 1, 40, 77, 128, 129, 200, 255]) == 0
        n = 4096
        b = W.make_batch_gpu(v, n, msg_sz=80, seed=0xc0, mix="c2")
        codes = torch.empty(n, dtype=torch.int8, device="cuda")
        torch.cuda.synchronize()
        v.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes, stream=CTX_STREAM)
        v.verify_dev(12, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes[:12], stream=CTX_STREAM)   # latency path
        v.sync()
        exp = O.verify_many(b.sigs.cpu().numpy(), b.pubs.cpu().numpy(), b.pool.cpu().numpy(),
                            b.msg_off.cpu().numpy().view(np.uint32), b.msg_sz.cpu().numpy().view(np.uint32))
        assert np.array_equal(codes.cpu().numpy(), exp)
        assert v.set_cu_mask(None) == 0
        v.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes, stream=CTX_STREAM)
        v.sync()
        assert np.array_equal(codes.cpu().numpy(), exp)
    finally:
        v.close()


def test_dsm_reserve_per_context_and_clamped():
    """fd_ed25519_hip_ctx_set_dsm_reserve: a reserve above half the resident
    DSM slots is clamped (returns 1) instead of leaving a one-workgroup grid
    (ADVICE r05), it applies to its context only, and the verdicts of a
    reserved context are the unreserved one's"""
    from firedancer_amd import Verifier
    from firedancer_amd.ed25519 import lib
    dev = torch.device("cuda", 0)
    a, b = Verifier(device=0, chunk_sigs=1 << 16), Verifier(device=0, chunk_sigs=1 << 16)
    try:
        assert lib().fd_ed25519_hip_ctx_set_dsm_reserve(a.ctx, 1 << 30) == 1
        assert lib().fd_ed25519_hip_ctx_set_dsm_reserve(a.ctx, 128) == 0
        n = 1 << 16
        x = W.make_batch_gpu(b, n, msg_sz=64, seed=0xd5a, mix="c2")
        ca = torch.zeros(n, dtype=torch.int8, device=dev)
        cb = torch.zeros(n, dtype=torch.int8, device=dev)
        a.verify_dev(n, x.sigs, x.pubs, x.pool, x.msg_off, x.msg_sz, ca)
        b.verify_dev(n, x.sigs, x.pubs, x.pool, x.msg_off, x.msg_sz, cb)
        torch.cuda.synchronize()
        assert torch.equal(ca, cb) and 0 < int((cb == 0).sum()) < n
    finally:
        a.close(); b.close()
