"""GPU: a block's sigverify through the reference's replay scheduler with
integration/fd_replay_hip.patch, on the engine (integration/sched_run.c,
"hip" mode: the patched fd_sched's bulk claims, packed into pinned buffers
and verified by fd_replay_hip_txn_verify_host, polled without blocking, as
the patched replay tile does).

- A 16384-txn block (1-12 signers, C2 mutations per signature, GPU-signed):
  every transaction's result equals the reference's own
  fd_executor_txn_verify (fd_ed25519_verify_batch_single_msg, compiled from
  its sources, run by the same driver in "exec" mode), transaction by
  transaction.
- A valid 16384-txn block completes with every signature verified on the
  GPU; a block with one bad signature is marked dead, abandoned and drained.
- fd_replay_hip_txn_verify_host on the same mixed block equals the
  reference's batch_single_msg per txn too (no scheduler in between).
Throughput of the block path: tools/replay_block_bench.py."""
import os

import numpy as np
import pytest

from replay_io import BUILD, block_fecs, block_stream, results_by_sig0, run_sched, write_block

pytestmark = pytest.mark.gpu
N = 16384


def _block(verifier, d, mix, seed, bad_at=None):
    from firedancer_amd.txn_workload import gpu_signer
    pool, off, sz, nsig = block_stream(N, gpu_signer(verifier), seed, mix, bad_at)
    path = str(d / f"block_{seed}.bin")
    write_block(path, block_fecs(pool, off, sz))
    return path, pool, off, sz, nsig


@pytest.fixture(scope="module")
def runs(verifier, tmp_path_factory):
    exe = os.path.join(BUILD, "sched_run_hip")
    assert os.path.exists(exe), f"{exe} missing: run __graft_entry__.build() in the build container"
    d = tmp_path_factory.mktemp("replay_gpu")
    mixed, mpool, moff, msz, msig = _block(verifier, d, "c2", 0x7e81)
    valid, _, voff, _, vsig = _block(verifier, d, "none", 0x7e82)
    bad, bpool, boff, _, _ = _block(verifier, d, "none", 0x7e83, bad_at=N // 2)
    jobs = {"mixed_exec": dict(block=mixed, mode="exec", exec_cnt=8, record=1),
            "mixed_hip": dict(block=mixed, mode="hip", exec_cnt=8, record=1, batch_max=4096, batch_min=256),
            "valid_hip": dict(block=valid, mode="hip", exec_cnt=8),
            "bad_hip": dict(block=bad, mode="hip", exec_cnt=8, batch_max=2048, batch_min=128)}
    res = dict(zip(jobs, run_sched("sched_run_hip", list(jobs.values()), d)))
    res["mixed"] = (mpool, moff, msz, msig)
    res["valid"] = (len(voff), vsig)
    res["bad_sig0"] = bpool[int(boff[N // 2]) + 1:int(boff[N // 2]) + 65].tobytes()
    return res


def test_block_equals_reference_txn_by_txn(runs):
    ie, re_ = runs["mixed_exec"]
    ih, rh = runs["mixed_hip"]
    for i in (ie, ih):
        assert i["block_ended"] == 1 and i["dead"] == 0 and i["refcnt"] == 0, i
    ref, got = results_by_sig0(re_), results_by_sig0(rh)
    n = len(runs["mixed"][1])
    assert n > 0.99 * N and len(ref) == n and len(got) == n
    diff = [k for k in ref if ref[k] != got[k]]
    assert not diff, len(diff)
    assert 0.3 < np.mean([v == 0 for v in ref.values()]) < 0.9
    assert ih["sigs_bulk"] > 0.9 * runs["mixed"][3] and ih["bulk_batches"] >= n // 4096, ih


def test_valid_block_all_on_gpu(runs):
    info, recs = runs["valid_hip"]
    assert info["block_ended"] == 1 and info["dead"] == 0 and info["refcnt"] == 0, info
    n, sigs = runs["valid"]
    assert info["sigverified"] == n and (recs["result"] == 0).all()
    assert info["sigs_bulk"] >= 0.9 * sigs, info


def test_bad_block_dies_on_gpu_verdict(runs):
    info, recs = runs["bad_hip"]
    assert info["dead"] == 1 and info["block_ended"] == 0, info
    got = results_by_sig0(recs)
    assert got.get(runs["bad_sig0"]) == -13 and sum(v != 0 for v in got.values()) == 1


def test_host_entry_point_equals_reference(runs, verifier):
    """fd_replay_hip_txn_verify_host over the mixed block (parse order of the
    oracle's parse), against the exec-mode reference results."""
    import txn_lib as T
    from firedancer_amd.replay import ReplayVerifier, descs_from_txn_t
    pool, off, sz, _ = runs["mixed"]
    n = len(off)
    tsz, out = T.oracle_parse_many(pool, off, sz)
    desc = descs_from_txn_t(out, off, sz)
    res = np.full(n, 7, np.int32)
    rv = ReplayVerifier(verifier, n)
    rv.txn_verify_host(n, np.ascontiguousarray(pool), desc, res)
    rv.wait()
    assert rv.poll() == 1
    rv.close()
    ref = results_by_sig0(runs["mixed_exec"][1])
    exp = np.array([ref[pool[int(o) + 1:int(o) + 65].tobytes()] for o in off], np.int32)
    assert np.array_equal(res, exp)
