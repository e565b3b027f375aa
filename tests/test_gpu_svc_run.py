"""GPU: the service-mode verify stage -- the reference's verify tiles with
integration/fd_verify_tile_svc.patch (no HIP in the tile processes) served by
the GPU tile (integration/svc_run.c: fd_verify_svc_* in
firedancer_amd/libfd_ed25519_hip.so, the requests of every tile merged into
one launch) -- in the reference's own run loop (integration/svc_tile_run.c).

- One tile (range mode, and the stem-polled form through the frag area):
  the published payloads in order (a digest), the outcome counts equal the
  reference tile's (oracle/tile_drv.c tile_drv_ref) on a generated stream
  with resends, grafted signatures, malformed payloads and bundles.
- Two tiles: each tile's published sequence equals the reference tile's
  over that tile's round robin share.
- At scale (2^18 GPU-signed C4 frags, two tiles): every tile's digest and
  counts equal the same stage with the CPU stand-in (oracle/_ref/svc_mock:
  the reference's own parse and verify behind the same protocol).
- A stalled consumer behind a 128-frag verify_dedup link with a third of the
  frags dropped: nothing overwritten, the reference's sequence.
- An unreliable producer (no flow control) far ahead of a shallow link: the
  lost frags are counted as the stem counts overruns, nothing aborts, every
  frag is accounted for.
- Every tile process: one thread, no /dev/kfd or /dev/dri fd after
  privileged_init."""
import os

import numpy as np
import pytest

import svc_io as S
import txn_lib as T
from tile_io import read_fdo1, run_driver, write_fdt1

pytestmark = pytest.mark.gpu

SEED, DEPTH = 0x5eed7117, 777
SMALL = {"SVC_RUN_SLOT_CAP": "1024", "SVC_RUN_REQ_DEPTH": "8"}


@pytest.fixture(scope="module")
def stream(tmp_path_factory):
    from firedancer_amd.txn_workload import make_txn_stream
    s = make_txn_stream(6000, T.oracle_signer, seed=0x7e65, dup_frac=0.05, graft_frac=0.01, bad_frac=0.02)
    bid = np.zeros(s.n, np.uint64)
    r = np.random.default_rng(0x7e66)
    for start in r.choice(s.n - 8, 60, replace=False):
        bid[start:start + int(r.integers(1, 6))] = int(r.integers(1, 2**40))
    d = tmp_path_factory.mktemp("svc")
    p = str(d / "stream.bin")
    write_fdt1(p, s.pool, s.off, s.sz, bid, SEED, DEPTH)
    run_driver("ref", p, str(d / "ref.bin"))
    return dict(path=p, s=s, bid=bid, ref=S.reference_digest(read_fdo1(str(d / "ref.bin"), DEPTH)))


def _check(r, n):
    assert r["overrun"] == 0 and r["lapped"] == 0 and r["consumer_bad"] == 0, r
    assert r["frags"] == n and r["consumed"] == r["published"]
    assert r["tile_threads_max"] == 1 and r["tile_dev_fds"] == 0
    assert r["metrics_ok"] == 1


@pytest.mark.parametrize("polled", [0, 1])
def test_one_tile_equals_reference_tile(stream, tmp_path, polled):
    env = dict(SMALL)
    if polled:
        env.update(SVC_RUN_POLLED="1", SVC_RUN_FRAG_CAP="512")
    r = S.run(stream["path"], 1, 1 << 14, str(tmp_path / "run"), env=env)
    _check(r, stream["s"].n)
    assert S.tile_counts(r["tiles"][0]) == stream["ref"]
    assert r["svc"]["launches"] >= 1 and r["svc"]["flushed_frags"] == r["published"]


def test_two_tiles_equal_reference_shares(stream, tmp_path):
    r = S.run(stream["path"], 2, 1 << 14, str(tmp_path / "run"), env=SMALL)
    _check(r, stream["s"].n)
    for t in range(2):
        p = str(tmp_path / f"share{t}.bin")
        S.share_stream(p, stream["s"], stream["bid"], t, 2, SEED, DEPTH)
        run_driver("ref", p, str(tmp_path / f"ref{t}.bin"))
        assert S.tile_counts(r["tiles"][t]) == S.reference_digest(read_fdo1(str(tmp_path / f"ref{t}.bin"), DEPTH)), t


def test_scale_equals_reference_code(tmp_path, verifier):
    import tile_bench as TB
    p = str(tmp_path / "c4.bin")
    s = TB.make_stream(1 << 18, p, seed=0x7e67)
    g = S.run(p, 2, 1 << 18, str(tmp_path / "gpu"), env={"SVC_RUN_PRELAY": "1"})
    m = S.run(p, 2, 1 << 18, str(tmp_path / "cpu"), env={"SVC_RUN_PRELAY": "1"}, mock=True, timeout=600)
    _check(g, s.n)
    _check(m, s.n)
    for t in range(2):
        assert S.tile_counts(g["tiles"][t]) == S.tile_counts(m["tiles"][t]), t
    assert g["sigs"] == m["sigs"] and g["published"] > 0.6 * s.n


def test_stalled_consumer_and_drops(tmp_path):
    from firedancer_amd.txn_workload import make_txn_stream
    s = make_txn_stream(3000, T.oracle_signer, seed=0x7e68, dup_frac=0.15, graft_frac=0.02, bad_frac=0.2)
    p = str(tmp_path / "s.bin")
    write_fdt1(p, s.pool, s.off, s.sz, np.zeros(s.n, np.uint64), SEED, DEPTH)
    run_driver("ref", p, str(tmp_path / "ref.bin"))
    ref = S.reference_digest(read_fdo1(str(tmp_path / "ref.bin"), DEPTH))
    r = S.run(p, 1, 1 << 14, str(tmp_path / "run"), env=dict(SMALL, SVC_RUN_CONS_STALL_MS="400", SVC_RUN_OUT_DEPTH="128"))
    _check(r, s.n)
    assert S.tile_counts(r["tiles"][0]) == ref
    assert r["regime"]["backpressure"] > 0.1


def test_unreliable_producer_overruns_are_dropped(tmp_path, verifier):
    import tile_bench as TB
    p = str(tmp_path / "c4.bin")
    s = TB.make_stream(1 << 18, p, seed=0x7e69)
    r = S.run(p, 1, 4096, str(tmp_path / "ovr"), env={"SVC_RUN_RATE": "200000000"})
    assert r["overrun"] + r["lapped"] > 0, r
    assert r["frags"] + r["overrun"] + r["lapped"] == s.n
    assert r["consumer_bad"] == 0 and r["tile_threads_max"] == 1 and r["metrics_ok"] == 1


def test_sandboxed_tiles_with_the_gpu_tile(stream, tmp_path):
    """the tiles inside the reference's fd_sandbox_enter (user namespace,
    pivot_root, landlock, the reference's seccomp policy) while the GPU tile
    serves them; skipped where user namespaces are refused"""
    import subprocess
    if subprocess.run(["unshare", "-U", "true"], capture_output=True).returncode:
        pytest.skip("user namespaces refused on this box")
    r = S.run(stream["path"], 2, 1 << 14, str(tmp_path / "run"), env=dict(SMALL, SVC_RUN_SANDBOX="1"))
    _check(r, stream["s"].n)
    assert all(x["sandboxed"] == 1 for x in r["tiles"])
    for t in range(2):
        p = str(tmp_path / f"share{t}.bin")
        S.share_stream(p, stream["s"], stream["bid"], t, 2, SEED, DEPTH)
        run_driver("ref", p, str(tmp_path / f"ref{t}.bin"))
        assert S.tile_counts(r["tiles"][t]) == S.reference_digest(read_fdo1(str(tmp_path / f"ref{t}.bin"), DEPTH)), t


@pytest.mark.parametrize("tiles", [1, 2])
def test_range_link_beside_a_polled_link(stream, tmp_path, tiles):
    """two quic_verify links, link 0 read by range and link 1 polled by the
    stem (frag requests): the order-free counts equal the reference's over
    each tile's share and the all-range run's (tests/test_svc_tile.py has
    the CPU stand-in's run of the same)"""
    s = stream["s"]
    p = str(tmp_path / "nobundle.bin")
    write_fdt1(p, s.pool, s.off, s.sz, np.zeros(s.n, np.uint64), SEED, 1 << 14)
    env = dict(SMALL, SVC_RUN_LINKS="2", SVC_RUN_FRAG_CAP="512")
    mixed = S.run(p, tiles, 1 << 14, str(tmp_path / "mixed"), env=dict(env, SVC_RUN_POLLED="2"))
    rng = S.run(p, tiles, 1 << 14, str(tmp_path / "range"), env=env)
    _check(mixed, s.n)
    _check(rng, s.n)

    def order_free(x):
        return (x["published"], x["parse_fail"], x["published"] + x["dedup"] + x["verify_fail"])
    for t in range(tiles):
        idx = np.array([j for j in range(s.n) if (j // 2) % tiles == t])
        ref = S.ref_share_digests(s.pool, s.off[idx], s.sz[idx], None, 1, SEED + t, 1 << 14)[0]
        assert order_free(mixed["tiles"][t]) == order_free(ref) == order_free(rng["tiles"][t]), t


def test_frags_shorter_than_their_payload_are_redone_on_the_tile(stream, tmp_path):
    """every 97th frag's mcache sz short of 80 + payload_sz: the GPU flags
    them (FD_VERIFY_SVC_RES_HOST) and the tile redoes them on its core, in
    order between the GPU's frags, on a 256-frag out link"""
    r = S.run(stream["path"], 1, 1 << 14, str(tmp_path / "run"), env=dict(SMALL, SVC_RUN_LIE="97", SVC_RUN_OUT_DEPTH="256"))
    _check(r, stream["s"].n)
    assert r["host_redone"] == len(range(96, stream["s"].n, 97))



def test_six_tiles_reference_default_topology(stream, tmp_path):
    """the reference's default verify_tile_count = 6 (default.toml:776) on one
    GPU, in the segment shape the topology gives it (fd_verify_svc_topo_shape:
    128 slots of 2048 frags, frag area 256; tests/test_svc_shape.py): each
    tile's published sequence equals the reference tile's over its share"""
    env = {"SVC_RUN_REQ_DEPTH": "128", "SVC_RUN_SLOT_CAP": "2048", "SVC_RUN_FRAG_CAP": "256"}
    r = S.run(stream["path"], 6, 1 << 14, str(tmp_path / "run"), env=env)
    _check(r, stream["s"].n)
    assert r["tile_cnt"] == 6 and r["req_depth"] == 128 and r["slot_cap"] == 2048
    for t in range(6):
        p = str(tmp_path / f"share{t}.bin")
        S.share_stream(p, stream["s"], stream["bid"], t, 6, SEED, DEPTH)
        run_driver("ref", p, str(tmp_path / f"ref{t}.bin"))
        assert S.tile_counts(r["tiles"][t]) == S.reference_digest(read_fdo1(str(tmp_path / f"ref{t}.bin"), DEPTH)), t
