"""GPU: ed25519 program instructions (fd_precompile_hip_ed25519_verify_dev)
against the oracle's restatement of fd_precompile_ed25519_verify
(oracle/fd_precompile_oracle.c; fd_precompiles.c:76-211) and against the
reference itself (compiled from its source, tests/test_precompile_ref.py), bit-exact in both
the return value and the custom error, on a synthetic block holding every
outcome class."""
import numpy as np
import pytest

import precompile_lib as P

pytestmark = pytest.mark.gpu


def _run(verifier, pool, desc, tab, max_instr=None):
    import torch
    from firedancer_amd.replay import PrecompileVerifier
    dev = torch.device("cuda", 0)
    n = desc.size
    pv = PrecompileVerifier(verifier, max_instr or n)
    err = torch.full((n,), 77, dtype=torch.int32, device=dev)
    ce = torch.full((n,), 77, dtype=torch.int32, device=dev)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).to(dev)
    pv.ed25519_verify_dev(n, t(pool), t(desc), t(tab if tab.size else np.zeros(1, P.PC_INSTR)), err, ce)
    out = err.cpu().numpy(), ce.cpu().numpy().view(np.uint32)
    pv.close()
    return out


def test_random_block_vs_oracle(verifier):
    pool, desc, tab = P.random_block(2024, 4000)
    err, ce = _run(verifier, pool, desc, tab)
    oerr, oce = P.oracle_many(pool, desc, tab)
    bad = np.nonzero((err != oerr) | (ce != oce))[0]
    assert bad.size == 0, [(int(j), int(err[j]), int(ce[j]), int(oerr[j]), int(oce[j])) for j in bad[:10]]
    assert set(oce.tolist()) == {0, 2, 3, 4}
    assert 0.3 < float((oce == 0).mean()) < 0.8


def test_descriptor_past_mtu_is_flagged(verifier):
    pool, desc, tab = P.random_block(7, 64)
    desc = desc.copy()
    desc[5]["data_sz"] = 1233
    err, ce = _run(verifier, np.concatenate([pool, np.zeros(1300, np.uint8)]), desc, tab)
    assert err[5] == -1 and ce[5] == 0xFFFFFFFF
    oerr, oce = P.oracle_many(pool, np.delete(desc, 5), tab)
    assert np.array_equal(np.delete(err, 5), oerr) and np.array_equal(np.delete(ce, 5), oce)


def test_batch_larger_than_max_instr_raises(verifier):
    import torch
    from firedancer_amd.replay import PrecompileVerifier
    pv = PrecompileVerifier(verifier, 4)
    z = torch.zeros(1024, dtype=torch.uint8, device="cuda:0")
    with pytest.raises(ValueError):
        pv.ed25519_verify_dev(5, z, z, z, z, z)
    pv.close()


def test_reference_fixture(verifier):
    """The GPU path against the reference's own fd_precompile_ed25519_verify
    (fd_precompiles.c:120-222, compiled from its source), through the committed
    answers of tests/golden/gen_precompile_ref.py; and against the compiled
    reference directly when oracle/_ref travelled with the tree."""
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "precompile_ref.npz"))
    pool, desc, tab = g["pool"], g["desc"].view(P.PC_DESC).reshape(-1), g["tab"].view(P.PC_INSTR).reshape(-1)
    err, ce = _run(verifier, pool, desc, tab)
    bad = np.nonzero((err != g["err"]) | (ce != g["custom_err"]))[0]
    assert bad.size == 0, [(int(j), int(err[j]), int(ce[j]), int(g["err"][j]), int(g["custom_err"][j]))
                           for j in bad[:10]]
    if os.path.exists(P.ref_path()):
        pool, desc, tab = P.random_block(31337, 1500)
        err, ce = _run(verifier, pool, desc, tab)
        rerr, rce = P.ref_many(pool, desc, tab)
        assert np.array_equal(err, rerr) and np.array_equal(ce, rce)
