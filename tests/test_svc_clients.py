"""CPU: the verify service's clients (include/fd_verify_svc.h "clients",
FD_VERIFY_SVC_REQ_SIGS) against the reference, with the GPU tile's CPU
stand-in (oracle/_ref/svc_mock: each record answered by the reference's own
fd_ed25519_verify).  The GPU half is tests/test_gpu_svc_clients.py.

The shred tile's FEC-set roots and the replay tile's block sigverify reach
the GPU through the per-GPU service as client tiles, so that both tiles keep
the reference's process model -- one thread, no device fd, the reference's
sandbox -- as the verify tiles do:

- the FEC resolver with integration/fd_fec_resolver_hip.patch in service
  mode (fd_fec_resolver_hip_attach_svc; integration/fec_run.c built with
  FD_HAS_HIP_SVC) gives every shred the reference add_shred's outcome and
  every completed set byte for byte (the same file as _build/fec_run_ref),
  takes the service's verdict for almost every first shred, and runs as one
  thread with no device fd;
- the replay scheduler with integration/fd_replay_hip.patch, its claimed
  batches verified as service records (include/fd_replay_svc.h;
  integration/sched_run.c svc mode), gives every transaction
  fd_executor_txn_verify's result on a block where ~40% fail, completes a
  valid block, and kills a block with one bad signature.
- the service rejects a client that posts a flush (a client has no out
  dcache) -- the mock's check, the GPU tile's is fd_verify_svc_poll's."""
import os

import pytest

import svc_io as SI
from replay_io import BUILD, results_by_sig0, run_sched_svc
from test_ref_replay import expected_exec, make_block

pytestmark = pytest.mark.skipif(not (os.path.exists(os.path.join(BUILD, "fec_run_svc")) and os.path.exists(SI.MOCK)),
                                reason="the client drivers need /root/reference (built by build())")


def _fec(tmp_path, window, sets=200, seed=0x5eedfec):
    import json
    import subprocess
    import svc_bench as SB
    svc = str(tmp_path / "svc.bin")
    r = SB.run_host([("fec", [os.path.join(BUILD, "fec_run_svc"), svc, str(sets), str(seed), str(window)])],
                    str(tmp_path / "logs"), svc_exe=SI.MOCK, timeout=240)
    ref = str(tmp_path / "ref.bin")
    p = subprocess.run([os.path.join(BUILD, "fec_run_ref"), ref, str(sets), str(seed), str(window)], capture_output=True,
                       text=True, timeout=240, check=True)
    return r, r["clients"]["fec"], json.loads(p.stdout.strip().splitlines()[-1]), open(svc, "rb").read(), open(ref, "rb").read()


@pytest.mark.parametrize("window", [64, 512])
def test_fec_roots_through_the_service_equal_reference(tmp_path, window):
    host, got, ref, gb, rb = _fec(tmp_path, window)
    assert got["hip"] == 2 and ref["hip"] == 0
    assert gb == rb
    for k in ("shreds", "sets", "rejected", "ignored", "okay", "completes"):
        assert got[k] == ref[k], k
    assert got["roots_checked"] == got["roots_verified"] > 0 and got["code_mismatch"] == 0 and got["code_diff"] == 0
    assert got["table_hits"] > 0 and got["core_verifies"] <= 0.01 * got["table_hits"]
    assert got["threads"] == 1 and got["dev_fds"] == 0
    assert host["svc"]["records"] == got["roots_verified"] and host["svc"]["requests"] == got["svc_requests"]


@pytest.fixture(scope="module")
def replay_runs(tmp_path_factory):
    d = tmp_path_factory.mktemp("replay_svc")
    mixed, mpool, moff, msz, mnsig = make_block(d, 1500, "c2", 0x7e91)
    valid, _, voff, _, _ = make_block(d, 700, "none", 0x7e92)
    bad, bpool, boff, _, _ = make_block(d, 900, "none", 0x7e93, bad_at=450)
    jobs = {"mixed": dict(block=mixed, mode="svc", record=1, batch_max=256, batch_min=32),
            "valid": dict(block=valid, mode="svc", exec_cnt=3, batch_max=128, batch_min=16),
            "bad": dict(block=bad, mode="svc", batch_max=64, batch_min=8)}
    res, host = run_sched_svc(list(jobs.values()), d, mock=True)
    out = dict(zip(jobs, res))
    out["host"] = host
    out["mixed_exp"] = expected_exec(mpool, moff, msz)
    out["mixed_n"], out["mixed_sigs"], out["valid_n"] = len(moff), mnsig, len(voff)
    out["bad_sig0"] = bpool[int(boff[450]) + 1:int(boff[450]) + 65].tobytes()
    return out


def test_replay_svc_every_txn_equals_reference(replay_runs):
    info, recs = replay_runs["mixed"]
    assert info["block_ended"] == 1 and info["dead"] == 0 and info["refcnt"] == 0, info
    assert results_by_sig0(recs) == replay_runs["mixed_exp"]
    assert info["sigs_bulk"] > 0.2 * replay_runs["mixed_sigs"] and info["svc_sigs"] == info["sigs_bulk"], info
    assert info["threads"] == 1 and info["dev_fds"] == 0, info


def test_replay_svc_valid_block_completes(replay_runs):
    info, recs = replay_runs["valid"]
    assert info["block_ended"] == 1 and info["dead"] == 0 and info["refcnt"] == 0, info
    assert info["sigverified"] == replay_runs["valid_n"] and (recs["result"] == 0).all()


def test_replay_svc_bad_signature_kills_the_block(replay_runs):
    info, recs = replay_runs["bad"]
    assert info["dead"] == 1 and info["block_ended"] == 0, info
    got = results_by_sig0(recs)
    assert got.get(replay_runs["bad_sig0"]) == -13
    assert sum(v != 0 for v in got.values()) == 1


def test_replay_tile_service_mode_has_no_hip():
    """integration/fd_replay_hip.patch with FD_HAS_HIP_SVC (_build/replay_tile_svc.o,
    -Wall -Wextra -Werror): the replay tile claims batches and joins the
    service as a client, and references nothing of the engine -- it keeps
    the reference's seccomp policy and fd list (its populate_allowed_*
    are the reference's in this build)"""
    import subprocess
    o = os.path.join(BUILD, "replay_tile_svc.o")
    assert os.path.exists(o)
    und = subprocess.run(["nm", "-u", o], capture_output=True, text=True, check=True).stdout
    assert "fd_sched_sigverify_claim" in und and "fd_sched_sigverify_claim_done" in und
    assert "hip" not in und.replace("fd_sched", ""), [x for x in und.split() if "hip" in x]


REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(REF), reason="needs /root/reference")
def test_shred_tile_patch_wires_the_burst(tmp_path):
    """integration/fd_shred_tile_hip.patch on src/disco/shred/fd_shred_tile.c
    (with the resolver patch): every line it adds sits in an FD_HAS_HIP_SVC
    block (without it the tile is the reference's, line for line); with it,
    the tile compiles -Wall -Wextra -Werror against the reference's headers,
    attaches its resolver to the GPU 0 service as a client
    (fd_fec_resolver_hip_attach_svc, memory from its scratch: the tile is
    sandboxed when it makes its resolver), and before add_shred on a shred
    of an unknown set (fd_fec_resolver_hip_needed) preverifies that shred
    with the frags already published after it on its net link
    (fd_fec_resolver_hip_preverify) -- and references nothing of the engine"""
    import shutil
    import subprocess
    from test_ref_tile import _strip_svc
    d = tmp_path / "src" / "disco" / "shred"
    os.makedirs(d)
    for f in ("fd_shred_tile.c", "fd_fec_resolver.c", "fd_fec_resolver.h"):
        shutil.copy(os.path.join(REF, "src/disco/shred", f), d / f)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in ("fd_shred_tile_hip.patch", "fd_fec_resolver_hip.patch"):
        subprocess.check_call(["patch", "-s", "-p1", "-i", os.path.join(repo, "integration", p)], cwd=tmp_path)
    got = open(d / "fd_shred_tile.c").read().splitlines()
    assert _strip_svc(got) == open(os.path.join(REF, "src/disco/shred/fd_shred_tile.c")).read().splitlines()
    body = "\n".join(got)
    for s_ in ("fd_fec_resolver_hip_attach_svc", "fd_fec_resolver_hip_needed", "fd_fec_resolver_hip_preverify",
               "fd_fec_resolver_hip_svc_footprint", "verify_svc.shred_client_base"):
        assert s_ in body, s_
    flags = ["gcc", "-std=c17", "-O1", "-DFD_HAS_HOSTED=1", "-DFD_HAS_INT128=1", "-DFD_HAS_DOUBLE=1", "-DFD_HAS_ALLOCA=1",
             "-DFD_HAS_X86=1", "-DFD_HAS_ATOMIC=1", "-DFD_HAS_THREADS=1", "-D_GNU_SOURCE", "-Wall", "-Wextra", "-Werror",
             "-I" + str(d), "-I" + os.path.join(REF, "src/disco/shred"), "-I" + os.path.join(repo, "include")]
    for svc in (0, 1):
        o = str(tmp_path / f"shred{svc}.o")
        subprocess.check_call(flags + ([f"-DFD_HAS_HIP_SVC=1"] if svc else []) + ["-c", str(d / "fd_shred_tile.c"), "-o", o])
        und = subprocess.run(["nm", "-u", o], capture_output=True, text=True, check=True).stdout
        assert ("fd_fec_resolver_hip_preverify" in und) == bool(svc) and ("fd_fec_resolver_hip_attach_svc" in und) == bool(svc)
        assert "fd_ed25519_hip" not in und
