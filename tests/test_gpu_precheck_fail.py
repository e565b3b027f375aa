"""GPU: batches in which (nearly) every record fails the pre-checks.

Round 3's fused prep+DSM kernel never returned on the 396-record
malleability set, most of whose records fail before the double-scalar
multiplication ("The k_verify_fused hang").  The shipped kernels
hand no work between workgroups inside a launch (k_verify_prep compacts
survivors through a device count, k_verify_dsm takes the count in its next
launch), and these sets check that a launch with few or no survivors ends
with the reference's codes: every record S >= L (fd_ed25519_user.c:150-152),
every record but five, and a small-order A on every other record, through
the bulk entry and through the replay block entry (segmented record counts,
k_msg_order over a nearly empty histogram).  Each runs once, like any other
test."""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu


def _batch(verifier, n, keep, seed):
    """n GPU-signed records over 64-byte messages; all but `keep` get S += L."""
    from firedancer_amd.workload import L_INT, SMALL_ORDER_ENCODINGS, make_batch_gpu
    b = make_batch_gpu(verifier, n, msg_sz=64, seed=seed, mix="c1")
    sigs, pubs = b.sigs.cpu().numpy().copy(), b.pubs.cpu().numpy().copy()
    pool, moff, msz = b.pool.cpu().numpy(), b.msg_off.cpu().numpy().view(np.uint32), b.msg_sz.cpu().numpy().view(np.uint32)
    rng = np.random.default_rng(seed)
    good = set(rng.choice(n, keep, replace=False).tolist()) if keep else set()
    so = np.frombuffer(b"".join(SMALL_ORDER_ENCODINGS), np.uint8).reshape(-1, 32)
    for i in range(n):
        if i in good:
            continue
        if i % 2:
            s = int.from_bytes(sigs[i, 32:].tobytes(), "little") + L_INT
            sigs[i, 32:] = np.frombuffer(s.to_bytes(32, "little"), np.uint8)
        else:
            pubs[i] = so[i % so.shape[0]]
    return sigs, pubs, pool, moff, msz, good


@pytest.mark.parametrize("n,keep", [(396, 0), (396, 5), (1 << 16, 0), (1 << 16, 5)])
def test_bulk_entry_few_survivors(verifier, n, keep):
    import torch
    sigs, pubs, pool, moff, msz, good = _batch(verifier, n, keep, 0x5e1 + n + keep)
    exp = O.verify_many(sigs, pubs, pool, moff, msz)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")  # noqa: E731
    codes = torch.full((n,), 9, dtype=torch.int8, device="cuda:0")
    verifier.verify_dev(n, t(sigs), t(pubs), t(pool), t(moff.view(np.int32)), t(msz.view(np.int32)), codes)
    verifier.sync()
    got = codes.cpu().numpy()
    assert np.array_equal(got, exp)
    assert int((got == 0).sum()) == keep


def test_replay_block_every_txn_fails(verifier):
    """A block of 4096 one-signature txns whose signatures all have S >= L:
    every txn gets FD_RUNTIME_TXN_ERR_SIGNATURE_FAILURE."""
    import torch
    from firedancer_amd.replay import DESC_DTYPE, ReplayVerifier
    n = 4096
    sigs, pubs, pool, moff, msz, _ = _batch(verifier, n, 0, 0x5e2)
    # txn j: [1][sig][message header 3 bytes][1 acct][pub][message 64 B]
    msg = pool[moff[:, None] + np.arange(64)]
    body = np.concatenate([np.ones((n, 1), np.uint8), sigs, np.tile(np.array([[1, 0, 0, 1]], np.uint8), (n, 1)),
                           pubs, msg], axis=1)
    desc = np.zeros(n, DESC_DTYPE)
    desc["payload_off"] = np.arange(n) * body.shape[1]
    desc["payload_sz"] = body.shape[1]
    desc["signature_off"], desc["signature_cnt"], desc["message_off"], desc["acct_addr_off"] = 1, 1, 65, 69
    rv = ReplayVerifier(verifier, n)
    res = torch.full((n,), 7, dtype=torch.int32, device="cuda:0")
    d_pool = torch.from_numpy(np.concatenate([body.reshape(-1), np.zeros(16, np.uint8)])).to("cuda:0")
    rv.txn_verify_dev(n, d_pool, torch.from_numpy(desc.view(np.uint8)).to("cuda:0"), res)
    verifier.sync()
    rv.close()
    assert bool((res == -13).all())
