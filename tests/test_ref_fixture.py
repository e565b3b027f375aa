"""CPU: the oracle against the reference-verdict fixtures at scale
(tests/golden/ref_scale_*.npz, made by tests/golden/gen_ref_scale.py from the
reference's own sign and verify), in both error modes: every record code and
every batch_single_msg group code."""
import os

import numpy as np
import pytest

import oracle_lib as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    d = np.load(os.path.join(GOLDEN, name))
    return {k: d[k] for k in d.files}


@pytest.mark.parametrize("mode,key", [(O.ERRMODE_AVX512, "code_avx512"), (O.ERRMODE_REF, "code_ref")])
def test_oracle_records_equal_reference(mode, key):
    r = _load("ref_scale_records.npz")
    got = O.verify_many(r["sigs"], r["pubs"], r["pool"], r["msg_off"], r["msg_sz"], mode)
    bad = np.nonzero(got != r[key])[0]
    assert bad.size == 0, [(int(i), int(got[i]), int(r[key][i]), int(r["extra"][i])) for i in bad[:10]]
    assert r["sigs"].shape[0] == 1 << 16


@pytest.mark.parametrize("mode,key", [(O.ERRMODE_AVX512, "gcode_avx512"), (O.ERRMODE_REF, "gcode_ref")])
def test_oracle_groups_equal_reference(mode, key):
    g = _load("ref_scale_groups.npz")
    sigs, pubs, pool = g["sigs"], g["pubs"], g["pool"]
    first, cnt, moff, msz = g["first"], g["cnt"], g["msg_off"], g["msg_sz"]
    # per-record codes once, then the batch semantics of user.c:232-310 on
    # the host -- and the oracle's own batch entry on a sample
    codes = O.verify_many(sigs, pubs, pool, moff, msz, mode)
    n = sigs.shape[0]
    for gi in range(first.size):
        f, c = int(first[gi]), int(cnt[gi])
        if c == 0 or c > 16:
            r = -1
        else:
            sc = codes[f:f + c]
            hard = sc[(sc == -1) | (sc == -2)]
            r = int(hard[0]) if hard.size else (-3 if (sc == -3).any() else 0)
        assert r == g[key][gi], (gi, r, int(g[key][gi]))
    rng = np.random.default_rng(3)
    for gi in rng.choice(first.size, 256, replace=False):
        f, c = int(first[gi]), int(cnt[gi])
        k = min(max(c, 1), n - f)
        m = pool[int(moff[f]):int(moff[f]) + int(msz[f])].tobytes()
        got = O.verify_batch_single_msg(m, sigs[f:f + k].tobytes(), pubs[f:f + k].tobytes(), c, mode)
        assert got == g[key][gi], (gi, got, int(g[key][gi]))
