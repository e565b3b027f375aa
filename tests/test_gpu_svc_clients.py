"""GPU: the shred tile's FEC-set roots and the replay tile's block sigverify
through the per-GPU verify service as client tiles (include/fd_verify_svc.h
"clients", FD_VERIFY_SVC_REQ_SIGS): the GPU tile (integration/svc_run.c,
inside its sandbox) verifies their signature records in its own launches;
the clients are the reference's resolver and scheduler built with
FD_HAS_HIP_SVC (integration/fec_run.c, integration/sched_run.c svc mode,
include/fd_replay_svc.h): no HIP in their processes.  VERDICT r05, next #4.

- FEC roots, windows of 64, 512 and 4096 shreds: every shred's add_shred
  outcome and every completed set byte-equal to the reference resolver's
  (_build/fec_run_ref); every root's verdict equals the reference's
  fd_ed25519_verify; add_shred takes the service's verdict for almost every
  first shred; the client is one thread with no device fd.
- Replay, 16384-txn GPU-signed blocks: every transaction's result equals
  the reference's fd_executor_txn_verify (sched_run_ref exec mode) on a
  block where ~40% fail; a valid block completes; one bad signature kills
  its block.
- Both at once beside the verify tiles: two verify tiles on a paced,
  unreliable quic_verify link of the reference's depth (16384) and a
  replay client posting a 16384-txn block into the same GPU tile: no frag
  lost, each tile's published sequence equal to the reference's over its
  share, every replay result equal to the reference's (the r05ah concern:
  another GPU user next to the verify stage -- here it is the same process's
  launches, so no second HIP process holds queues on the card)."""
import json
import os
import subprocess

import numpy as np
import pytest

import svc_io as S
from replay_io import BUILD, block_fecs, block_stream, results_by_sig0, run_sched, run_sched_svc, \
    sched_jobs_file, write_block

pytestmark = pytest.mark.gpu
N = 16384


def _fec(tmp_path, window, sets=1024):
    import svc_bench as SB
    seed = 0x5eedfec + window
    svc = str(tmp_path / "svc.bin")
    r = SB.run_host([("fec", [os.path.join(BUILD, "fec_run_svc"), svc, str(sets), str(seed), str(window)])],
                    str(tmp_path / "logs"), timeout=300)
    ref = str(tmp_path / "ref.bin")
    p = subprocess.run([os.path.join(BUILD, "fec_run_ref"), ref, str(sets), str(seed), str(window)], capture_output=True,
                       text=True, timeout=300, check=True)
    return r, r["clients"]["fec"], json.loads(p.stdout.strip().splitlines()[-1]), open(svc, "rb").read(), open(ref, "rb").read()


@pytest.mark.parametrize("window", [64, 512, 4096])
def test_fec_roots_through_the_gpu_service(tmp_path, window):
    host, got, ref, gb, rb = _fec(tmp_path, window)
    print(json.dumps({"window": window, "svc": got, "host": host}))
    assert got["hip"] == 2 and ref["hip"] == 0
    assert gb == rb
    for k in ("shreds", "sets", "rejected", "ignored", "okay", "completes"):
        assert got[k] == ref[k], k
    assert got["roots_checked"] == got["roots_verified"] > 0 and got["code_mismatch"] == 0
    assert got["table_hits"] > 0 and got["core_verifies"] <= 0.01 * got["table_hits"]
    assert got["threads"] == 1 and got["dev_fds"] == 0
    assert host["svc_sandboxed"] == 1 and host["svc"]["records"] == got["roots_verified"]


def _block(verifier, d, mix, seed, bad_at=None):
    from firedancer_amd.txn_workload import gpu_signer
    pool, off, sz, nsig = block_stream(N, gpu_signer(verifier), seed, mix, bad_at)
    path = str(d / f"block_{seed}.bin")
    write_block(path, block_fecs(pool, off, sz))
    return path, pool, off, sz, nsig


@pytest.fixture(scope="module")
def blocks(verifier, tmp_path_factory):
    d = tmp_path_factory.mktemp("replay_svc_gpu")
    mixed, mpool, moff, msz, msig = _block(verifier, d, "c2", 0x7e81)
    valid, _, voff, _, vsig = _block(verifier, d, "none", 0x7e82)
    bad, bpool, boff, _, _ = _block(verifier, d, "none", 0x7e83, bad_at=N // 2)
    ref = dict(zip(["mixed_exec"], run_sched("sched_run_ref", [dict(block=mixed, mode="exec", exec_cnt=8, record=1)], d)))
    return dict(d=d, mixed=mixed, valid=valid, bad=bad, mixed_n=len(moff), mixed_sigs=msig, valid_n=len(voff), valid_sigs=vsig,
                bad_sig0=bpool[int(boff[N // 2]) + 1:int(boff[N // 2]) + 65].tobytes(),
                ref=results_by_sig0(ref["mixed_exec"][1]))


@pytest.fixture(scope="module")
def replay_runs(blocks, tmp_path_factory):
    d = tmp_path_factory.mktemp("replay_svc_runs")
    jobs = {"mixed": dict(block=blocks["mixed"], mode="svc", exec_cnt=8, record=1, batch_max=4096, batch_min=256),
            "valid": dict(block=blocks["valid"], mode="svc", exec_cnt=8),
            "bad": dict(block=blocks["bad"], mode="svc", exec_cnt=8, batch_max=2048, batch_min=128)}
    res, host = run_sched_svc(list(jobs.values()), d)
    out = dict(zip(jobs, res))
    out["host"] = host
    return out


def test_replay_block_through_the_gpu_service(blocks, replay_runs):
    info, recs = replay_runs["mixed"]
    print(json.dumps({"mixed": info, "host": replay_runs["host"]}))
    assert info["block_ended"] == 1 and info["dead"] == 0 and info["refcnt"] == 0, info
    got, ref = results_by_sig0(recs), blocks["ref"]
    assert len(got) == len(ref) == blocks["mixed_n"]
    assert not [k for k in ref if ref[k] != got[k]]
    assert 0.3 < np.mean([v == 0 for v in ref.values()]) < 0.9
    assert info["sigs_bulk"] > 0.9 * blocks["mixed_sigs"] and info["svc_sigs"] == info["sigs_bulk"], info
    assert info["threads"] == 1 and info["dev_fds"] == 0, info
    assert replay_runs["host"]["svc_sandboxed"] == 1


def test_replay_valid_and_bad_blocks_through_the_gpu_service(blocks, replay_runs):
    info, recs = replay_runs["valid"]
    assert info["block_ended"] == 1 and info["dead"] == 0 and info["refcnt"] == 0, info
    assert info["sigverified"] == blocks["valid_n"] and (recs["result"] == 0).all()
    assert info["sigs_bulk"] >= 0.9 * blocks["valid_sigs"], info
    info, recs = replay_runs["bad"]
    assert info["dead"] == 1 and info["block_ended"] == 0, info
    got = results_by_sig0(recs)
    assert got.get(blocks["bad_sig0"]) == -13 and sum(v != 0 for v in got.values()) == 1


def test_replay_beside_verify_tiles_at_the_reference_depth(blocks, tmp_path):
    import svc_bench as SB
    import tile_bench as TB
    tiles, depth, rate = 2, 16384, 3000000
    p = str(tmp_path / "c4.bin")
    s = TB.make_stream(1 << 19, p, seed=0x7e6b)
    jf, outs = sched_jobs_file([dict(block=blocks["mixed"], mode="svc", exec_cnt=8, record=1, batch_max=4096,
                                     batch_min=256)], tmp_path)
    env = {"SVC_RUN_PRELAY": "1", "SVC_RUN_REQ_DEPTH": "128", "SVC_RUN_SLOT_CAP": "2048", "SVC_RUN_RATE": str(rate),
           "SVC_RUN_DIGEST": "1"}
    r = SB.run_one(p, tiles, depth, 400, str(tmp_path / "logs"), env=env, pin="auto",
                   clients=[("replay", [os.path.join(BUILD, "sched_run_svc"), jf])])
    lost = r["overrun"] + r["lapped"] + r.get("unseen", 0)
    print(json.dumps({"frags_per_s": r["frags_per_s"], "lost": lost, "latency": r["latency"],
                      "replay": r["clients"]["replay"]}))
    assert lost == 0 and r["frags"] == s.n and r["consumer_bad"] == 0, r
    assert r["tile_threads_max"] == 1 and r["tile_dev_fds"] == 0
    ref = S.ref_share_digests(s.pool, s.off, s.sz, None, tiles, 0x7f4a11, 4194302, threads=16)
    assert [S.tile_counts(x) for x in r["tiles"]] == [{k: x[k] for k in S.tile_counts(r["tiles"][0])} for x in ref]
    from replay_io import read_records
    info = json.loads([x for x in r["clients_lines"]["replay"] if x.startswith("{")][-1])
    assert info["block_ended"] == 1 and info["dead"] == 0 and info["threads"] == 1 and info["dev_fds"] == 0, info
    got = results_by_sig0(read_records(outs[0]))
    assert got == blocks["ref"]
