"""GPU: the service-mode GPU tile inside its sandbox (include/fd_hip_tile_sandbox.h
fd_hip_tile_sandbox_process, entered by integration/svc_run.c once the service
runs, as integration/fd_verify_gpu_tile.c enters it in unprivileged_init).

The reference runs every tile through fd_sandbox_enter (src/disco/topo/
fd_topo_run.c:122).  A process that owns a HIP context has the runtime's
threads, so the user namespace and pivot_root are out of reach
(fd_sandbox.c:649); the rest applies to every thread: the fd allow-list,
rlimits, no capabilities, no_new_privs, and a seccomp filter installed with
SECCOMP_FILTER_FLAG_TSYNC (missing #1: the process that reads
every quic_verify frag and writes every tile's out dcache had none).

- every thread of the GPU tile has Seccomp 2 and NoNewPrivs 1 while it
  serves two tiles, and the tiles' published sequences equal the reference
  tile's over their shares;
- with SECCOMP_RET_TRAP as the filter's action the same run traps no call:
  the allow list covers what the runtime and the service do, teardown
  included;
- a refused call (getppid, right after entering) kills the process: SIGSYS."""
import signal

import pytest

import svc_io as S
from tile_io import read_fdo1, run_driver
from test_gpu_svc_run import DEPTH, SEED, SMALL, _check, stream  # noqa: F401  (the module's stream fixture)

pytestmark = pytest.mark.gpu


def _two_tiles_equal(r, stream, tmp_path):
    for t in range(2):
        p = str(tmp_path / f"share{t}.bin")
        S.share_stream(p, stream["s"], stream["bid"], t, 2, SEED, DEPTH)
        run_driver("ref", p, str(tmp_path / f"ref{t}.bin"))
        assert S.tile_counts(r["tiles"][t]) == S.reference_digest(read_fdo1(str(tmp_path / f"ref{t}.bin"), DEPTH)), t


def test_every_gpu_tile_thread_is_filtered(stream, tmp_path):
    r = S.run(stream["path"], 2, 1 << 14, str(tmp_path / "run"), env=dict(SMALL), svc_env={"SVC_SANDBOX": "kill"})
    _check(r, stream["s"].n)
    sb = r["svc_sandbox"]
    assert sb["sandboxed"] == 1 and sb["traps"] == 0, sb
    assert sb["threads"] >= 2 and sb["seccomp_threads"] == sb["threads"] and sb["nnp_threads"] == sb["threads"], sb
    _two_tiles_equal(r, stream, tmp_path)


def test_trap_mode_traps_nothing(stream, tmp_path):
    r = S.run(stream["path"], 2, 1 << 14, str(tmp_path / "run"), env=dict(SMALL), svc_env={"SVC_SANDBOX": "trap"})
    _check(r, stream["s"].n)
    sb = r["svc_sandbox"]
    assert sb["sandboxed"] == 1 and sb["traps"] == 0 and sb["trap_nr"] == [], sb


def test_refused_call_kills_the_gpu_tile(stream, tmp_path):
    with pytest.raises(RuntimeError) as e:
        S.run(stream["path"], 1, 1 << 14, str(tmp_path / "run"), env=dict(SMALL),
              svc_env={"SVC_SANDBOX": "kill", "SVC_SANDBOX_PROBE": "1"}, timeout=120)
    assert f"('svc', {-signal.SIGSYS})" in str(e.value), str(e.value)
