"""GPU parity of the replay and shred callers (include/fd_replay_hip.h) against
the oracle restatement: fd_executor_txn_verify over whole blocks of parsed
transactions (fd_executor.c:1607-1623), its batch_sz edge cases, and the FEC
resolver's 32-byte root check (fd_fec_resolver.c:476).  Bit-exact."""
import numpy as np
import pytest

import oracle_lib as O
import txn_lib as T

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch
    a = np.ascontiguousarray(a)
    if a.size == 0:
        a = np.zeros(1, a.dtype)
    return torch.from_numpy(a).to("cuda:0")


def _expected_exec(pool, desc):
    """fd_executor_txn_verify restated on the oracle, one txn at a time."""
    out = np.zeros(desc.size, np.int32)
    for j, d in enumerate(desc):
        p = pool[int(d["payload_off"]):int(d["payload_off"]) + int(d["payload_sz"])]
        so, mo, ao, cnt = int(d["signature_off"]), int(d["message_off"]), int(d["acct_addr_off"]), int(d["signature_cnt"])
        if cnt == 0 or cnt > 16:
            code = O.verify_batch_single_msg(p[mo:].tobytes(), b"\0" * 64, b"\0" * 32, cnt & 0xff)
        else:
            code = O.verify_batch_single_msg(p[mo:].tobytes(), p[so:so + 64 * cnt].tobytes(),
                                             p[ao:ao + 32 * cnt].tobytes(), cnt)
        out[j] = 0 if code == 0 else -13
    return out


def _run_replay(verifier, pool, desc, max_txn=None):
    import torch
    from firedancer_amd.replay import ReplayVerifier
    n = desc.size
    rv = ReplayVerifier(verifier, max_txn or max(n, 1))
    d_pool = _dev(np.concatenate([pool, np.zeros(16, np.uint8)]))
    d_desc = _dev(desc.view(np.uint8))
    d_res = torch.full((max(n, 1),), 7, dtype=torch.int32, device="cuda:0")
    rv.txn_verify_dev(n, d_pool, d_desc, d_res)
    verifier.sync()
    res = d_res.cpu().numpy()[:n]
    rv.close()
    return res


def test_replay_block_vs_oracle(verifier):
    """A 3000-txn block (1-12 signers, C2 mutations per signature) parsed by
    the oracle's fd_txn_parse, verified as fd_executor_txn_verify would."""
    from firedancer_amd.replay import descs_from_txn_t
    from firedancer_amd.txn_workload import make_txn_stream
    s = make_txn_stream(3000, T.oracle_signer, seed=0x5150, dup_frac=0.0, graft_frac=0.0, bad_frac=0.0)
    tsz, out = T.oracle_parse_many(s.pool, s.off, s.sz)
    ok = np.nonzero(tsz)[0]
    desc = descs_from_txn_t(out[ok], s.off[ok], s.sz[ok])
    exp = _expected_exec(s.pool, desc)
    got = _run_replay(verifier, s.pool, desc)
    assert np.array_equal(got, exp)
    assert 0.3 < (got == 0).mean() < 0.95 and (got == -13).any()
    assert (desc["signature_cnt"] > 1).sum() > 100


def test_replay_batch_sz_edges(verifier):
    """signature_cnt 0, 1, 16 (all valid), 16 (one bad), 17 (ERR_SIG unread)."""
    rng = np.random.default_rng(3)
    msg = rng.integers(0, 256, 100, dtype=np.uint8)
    prvs = rng.integers(0, 256, (17, 32), dtype=np.uint8)
    mpool = np.concatenate([msg, np.zeros(16, np.uint8)])
    pubs, sigs = O.sign_many(prvs, mpool, np.zeros(17, np.uint32), np.full(17, 100, np.uint32))
    payload = np.concatenate([sigs.reshape(-1), pubs.reshape(-1), msg])
    bad = payload.copy()
    bad[64 * 9 + 5] ^= 0x10                                  # signature 9 of 16
    pool = np.concatenate([payload, bad])
    from firedancer_amd.replay import DESC_DTYPE
    rows = []
    for off, cnt in ((0, 0), (0, 1), (0, 16), (payload.size, 16), (0, 17), (0, 255)):
        d = np.zeros(1, DESC_DTYPE)
        d["payload_off"], d["payload_sz"], d["signature_cnt"] = off, payload.size, cnt
        d["signature_off"], d["acct_addr_off"], d["message_off"] = 0, 64 * 17, 96 * 17
        rows.append(d)
    desc = np.concatenate(rows)
    exp = _expected_exec(pool, desc)
    assert exp.tolist() == [-13, 0, 0, -13, -13, -13]
    assert np.array_equal(_run_replay(verifier, pool, desc), exp)
    assert _run_replay(verifier, pool, desc[:0], max_txn=4).size == 0


def test_replay_max_txn_guard(verifier):
    import torch
    from firedancer_amd.replay import DESC_DTYPE, ReplayVerifier
    rv = ReplayVerifier(verifier, 4)
    d = torch.zeros(16 * 8, dtype=torch.uint8, device="cuda:0")
    with pytest.raises(ValueError):
        rv.txn_verify_dev(8, d, d, d)
    rv.close()
    assert DESC_DTYPE.itemsize == 16


def test_replay_host_entry_rejects_bad_spans(verifier):
    """fd_replay_hip_txn_verify_host refuses (nothing launched) a descriptor
    whose payload runs past pool_sz, n over max_txn, and a pool over its
    staging; a good call after them still verifies."""
    from firedancer_amd.replay import DESC_DTYPE, ReplayVerifier
    rv = ReplayVerifier(verifier, 4)
    pool = np.zeros(300, np.uint8)
    desc = np.zeros(2, DESC_DTYPE)
    desc["payload_off"], desc["payload_sz"], desc["signature_cnt"] = [0, 200], [150, 150], 1
    res = np.zeros(2, np.int32)
    with pytest.raises(ValueError):
        rv.txn_verify_host(2, pool, desc, res)                       # 200 + 150 > 300
    with pytest.raises(ValueError):
        rv.txn_verify_host(5, np.zeros(5 * 1232, np.uint8), np.zeros(5, DESC_DTYPE), np.zeros(5, np.int32))
    with pytest.raises(ValueError):
        rv.txn_verify_host(1, np.zeros(4 * 1232 + 1, np.uint8), desc[:1], res[:1])
    desc["payload_off"][1] = 150
    rv.txn_verify_host(2, pool, desc, res)
    rv.wait()
    assert (res == -13).all()                                       # zero signatures over zero keys
    rv.close()


def test_fec_roots_vs_oracle(verifier):
    """5000 FEC-set roots signed by 4 leaders, C2 mutations, through the
    fixed-size-message path; codes equal the oracle's fd_ed25519_verify."""
    import torch
    from firedancer_amd.replay import fec_verify_roots_dev
    from firedancer_amd.workload import c2_mutate
    rng = np.random.default_rng(11)
    n = 5000
    roots = rng.integers(0, 256, n * 32, dtype=np.uint8)
    leaders = rng.integers(0, 256, (4, 32), dtype=np.uint8)
    prvs = leaders[rng.integers(0, 4, n)]
    moff = (np.arange(n) * 32).astype(np.uint32)
    msz = np.full(n, 32, np.uint32)
    pool = np.concatenate([roots, np.zeros(16, np.uint8)])
    pubs, sigs = O.sign_many(prvs, pool, moff, msz)
    assert len(np.unique(pubs, axis=0)) == 4
    c2_mutate(sigs, pubs, rng)
    exp = O.verify_many(sigs, pubs, pool, moff, msz)
    codes = torch.zeros(n, dtype=torch.int8, device="cuda:0")
    fec_verify_roots_dev(verifier, n, _dev(pool), _dev(sigs), _dev(pubs), codes)
    verifier.sync()
    got = codes.cpu().numpy()
    assert np.array_equal(got, exp)
    assert 0.6 < (got == 0).mean() < 0.95


def test_fixed_matches_offsets(verifier):
    """verify_fixed_dev(msg_sz) == verify_dev with explicit offsets, across
    several chunks (the verifier fixture's chunk is 2^18)."""
    import torch
    from firedancer_amd.workload import make_batch_gpu
    n = (1 << 18) + 777
    b = make_batch_gpu(verifier, n, msg_sz=64, seed=77, mix="c2")
    c1 = torch.zeros(n, dtype=torch.int8, device="cuda:0")
    c2 = torch.zeros(n, dtype=torch.int8, device="cuda:0")
    verifier.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, c1)
    verifier.verify_fixed_dev(n, b.sigs, b.pubs, b.pool, 64, c2)
    verifier.sync()
    assert torch.equal(c1, c2)
    assert 0.7 < float((c1 == 0).float().mean()) < 0.9


def test_verify_dev_count(verifier):
    """verify_dev_count: records [0, *d_n) verified exactly as verify_dev,
    codes past the device-side count untouched; n_max spans three chunks of
    the fixture's 2^18 (counts ending inside the second chunk, inside the
    first, and zero).  Buffers hold n_max records (the host cannot see *d_n)."""
    import torch
    n = 3 << 18
    from firedancer_amd.workload import make_batch_gpu
    b = make_batch_gpu(verifier, n, msg_sz=48, seed=91, mix="c2")
    ref = torch.zeros(n, dtype=torch.int8, device="cuda:0")
    verifier.verify_dev(n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, ref)
    for cnt in (n, (1 << 18) + 4000, (1 << 18) + 17, 1000, 0):
        d_n = torch.tensor([cnt], dtype=torch.int32, device="cuda:0")
        codes = torch.full((n,), 5, dtype=torch.int8, device="cuda:0")
        bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda:0")
        verifier.verify_dev_count(n, d_n, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes, bm)
        verifier.sync()
        assert torch.equal(codes[:cnt], ref[:cnt]), cnt
        assert bool((codes[cnt:] == 5).all()), cnt
        bits = np.unpackbits(bm.cpu().numpy().view(np.uint8), bitorder="little")[:cnt].astype(bool)
        assert np.array_equal(bits, ref[:cnt].cpu().numpy() == 0), cnt


def test_device_entry_points_reject_bad_buffers(verifier):
    """Host arrays, short tensors and non-contiguous tensors are refused
    before any launch (they would fault or read out of bounds on the GPU)."""
    import torch
    n = 1024
    d = lambda k: torch.zeros(k, dtype=torch.uint8, device="cuda:0")  # noqa: E731
    good = dict(sigs=d(64 * n), pubs=d(32 * n), pool=d(64), msg_off=d(4 * n), msg_sz=d(4 * n), codes=d(n))
    args = lambda **kw: [kw.get(k, v) for k, v in good.items()]  # noqa: E731
    with pytest.raises(TypeError):
        verifier.verify_dev(n, *args(sigs=np.zeros(64 * n, np.uint8)))
    with pytest.raises(ValueError):
        verifier.verify_dev(n, *args(pubs=d(32 * n - 1)))
    with pytest.raises(ValueError):
        verifier.verify_dev(n, *args(codes=d(2 * n)[::2]))
    with pytest.raises(ValueError):
        verifier.verify_dev(n, *args(), bitmap=d(8))
