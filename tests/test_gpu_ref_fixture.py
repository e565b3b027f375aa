"""GPU: the engine against the reference's own verdicts at scale, from
committed fixtures (tests/golden/gen_ref_scale.py: signed by the reference's
fd_ed25519_sign, verdicts from the reference's fd_ed25519_verify /
fd_ed25519_verify_batch_single_msg, AVX-512 IFMA and portable backends,
src/ballet/ed25519/fd_ed25519_user.c:135-310).

Nothing here needs the reference or oracle/_ref on the GPU box, so these
tests never skip for a missing binary.  Every record / group code must equal
the reference's, in both error modes, through:
  - the bulk device entry (fd_ed25519_hip_verify_dev, codes + bitmap),
  - the host-memory entry (fd_ed25519_hip_verify_host),
  - the group reduce (k_group_reduce over per-record codes),
  - the drop-in fd_ed25519_verify_batch_single_msg for every group and the
    drop-in fd_ed25519_verify for a sample of records (long messages
    included)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def _load(name):
    d = np.load(os.path.join(GOLDEN, name))     # allow_pickle=False (default)
    return {k: d[k] for k in d.files}


@pytest.fixture(scope="module")
def recs():
    return _load("ref_scale_records.npz")


@pytest.fixture(scope="module")
def grps():
    return _load("ref_scale_groups.npz")


def _dev(verifier, a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(torch.device("cuda", verifier.device))


def _verify_dev(verifier, r, mode):
    import torch
    n = r["sigs"].shape[0]
    t = lambda a: _dev(verifier, a)
    codes = torch.zeros(n, dtype=torch.int8, device=torch.device("cuda", verifier.device))
    bitmap = torch.zeros((n + 63) // 64, dtype=torch.int64, device=codes.device)
    verifier.set_errmode(mode)
    try:
        verifier.verify_dev(n, t(r["sigs"]), t(r["pubs"]), t(r["pool"]), t(r["msg_off"].view(np.int32)),
                            t(r["msg_sz"].view(np.int32)), codes, bitmap)
        verifier.sync()
    finally:
        from firedancer_amd import ERRMODE_AVX512
        verifier.set_errmode(ERRMODE_AVX512)
    return codes.cpu().numpy(), bitmap.cpu().numpy()


def _mismatch(got, exp, extra=None):
    bad = np.nonzero(got != exp)[0]
    return bad.size, [(int(i), int(got[i]), int(exp[i])) + ((int(extra[i]),) if extra is not None else ())
                      for i in bad[:10]]


@pytest.mark.parametrize("mode_name", ["avx512", "ref"])
def test_records_bulk_equal_reference(verifier, recs, mode_name):
    from firedancer_amd import ERRMODE_AVX512, ERRMODE_REF
    mode = ERRMODE_AVX512 if mode_name == "avx512" else ERRMODE_REF
    exp = recs[f"code_{mode_name}"]
    got, bitmap = _verify_dev(verifier, recs, mode)
    assert np.array_equal(got, exp), _mismatch(got, exp, recs["extra"])
    n = exp.size
    bits = np.unpackbits(bitmap.view(np.uint8), bitorder="little")[:n].astype(bool)
    assert np.array_equal(bits, exp == 0)
    # every verdict class and every mutation class is present in the fixture
    assert set(np.unique(exp).tolist()) == {0, -1, -2, -3}
    assert set(np.unique(recs["extra"]).tolist()) == set(range(11))


def test_records_host_entry_equal_reference(verifier, recs):
    n = 8192                                           # a slice through the host-memory entry
    sl = slice(0, n)
    moff = recs["msg_off"][sl]; msz = recs["msg_sz"][sl]
    lo = int(moff.min()); hi = int((moff.astype(np.int64) + msz).max())
    pool = recs["pool"][lo:hi]
    codes, bitmap = verifier.verify_host(recs["sigs"][sl], recs["pubs"][sl], pool, (moff - lo).astype(np.uint32), msz)
    exp = recs["code_avx512"][sl]
    assert np.array_equal(codes, exp), _mismatch(codes, exp)
    bits = np.unpackbits(bitmap.view(np.uint8), bitorder="little")[:n].astype(bool)
    assert np.array_equal(bits, exp == 0)


@pytest.mark.parametrize("mode_name", ["avx512", "ref"])
def test_groups_equal_reference(verifier, grps, mode_name):
    import torch
    from firedancer_amd import ERRMODE_AVX512, ERRMODE_REF
    mode = ERRMODE_AVX512 if mode_name == "avx512" else ERRMODE_REF
    codes, _ = _verify_dev(verifier, grps, mode)
    ng = grps["first"].size
    out = torch.zeros(ng, dtype=torch.int8, device=torch.device("cuda", verifier.device))
    verifier.group_reduce_dev(ng, _dev(verifier, grps["first"].view(np.int32)), _dev(verifier, grps["cnt"]),
                              _dev(verifier, codes), out)
    verifier.sync()
    got = out.cpu().numpy()
    exp = grps[f"gcode_{mode_name}"]
    assert np.array_equal(got, exp), _mismatch(got, exp)
    assert set(np.unique(exp).tolist()) == {0, -1, -2, -3}


def test_groups_dropin_equal_reference(grps):
    """fd_ed25519_verify_batch_single_msg (the drop-in, process default
    context, AVX-512 codes) for every group of the fixture."""
    from firedancer_amd import fd_ed25519_verify_batch_single_msg
    sigs, pubs, pool = grps["sigs"], grps["pubs"], grps["pool"]
    first, cnt, moff, msz = grps["first"], grps["cnt"], grps["msg_off"], grps["msg_sz"]
    nrec = sigs.shape[0]
    got = np.zeros(first.size, np.int8)
    for g in range(first.size):
        f, c = int(first[g]), int(cnt[g])
        m = pool[int(moff[f]):int(moff[f]) + int(msz[f])].tobytes()
        k = min(max(c, 1), nrec - f)                   # the records the call may read (17: one past the group)
        got[g] = fd_ed25519_verify_batch_single_msg(m, sigs[f:f + k].tobytes(), pubs[f:f + k].tobytes(), c)
    exp = grps["gcode_avx512"]
    assert np.array_equal(got, exp), _mismatch(got, exp)


def test_records_dropin_single_equal_reference(recs):
    """fd_ed25519_verify (the drop-in) on a sample: 16 records of every
    verdict x mutation class present, and every long message."""
    from firedancer_amd import fd_ed25519_verify
    rng = np.random.default_rng(7)
    exp = recs["code_avx512"]
    pick = set(np.nonzero(recs["msg_sz"] > 1232)[0].tolist())
    for c in np.unique(exp):
        for x in np.unique(recs["extra"]):
            ix = np.nonzero((exp == c) & (recs["extra"] == x))[0]
            pick.update(rng.choice(ix, min(16, ix.size), replace=False).tolist())
    pick = np.array(sorted(pick))
    got = np.array([fd_ed25519_verify(recs["pool"][int(recs["msg_off"][i]):int(recs["msg_off"][i]) +
                                                   int(recs["msg_sz"][i])].tobytes(),
                                      recs["sigs"][i].tobytes(), recs["pubs"][i].tobytes()) for i in pick], np.int8)
    assert np.array_equal(got, exp[pick]), _mismatch(got, exp[pick])
    assert pick.size > 300
