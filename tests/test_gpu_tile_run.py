"""GPU: the patched reference verify tile in the reference's own run loop
(integration/tile_run.c: fd_verify_tile.c + integration/fd_verify_tile_hip.patch
in stem_run1, a producer process on the quic_verify link), as the bench's
tile leg runs it.

- The GPU-side during_frag (the patch's default) and the reference's host
  copy (FD_VERIFY_HIP_GPU_COPY 0) give the same outcome counts -- published,
  parse / verify / dedup / bundle failures and signatures -- over a C4
  stream (one tile: arrival order, and so the tcache's dedup decisions, is
  the link's seq order in both).
- With the producer allowed to run a whole link depth past the tile's
  consumption (TILE_RUN_NO_MARGIN) and a link shallower than the frags the
  GPU-copy tile holds unread, frags are overwritten before the GPU reads
  them: the tile drops them as overruns (fd_verify_hip_tile_complete_skip)
  and keeps running -- every frag is either an outcome or an overrun, and
  nothing aborts on the overwritten bytes.
- Range mode (TILE_RUN_RANGE: the tiles' quic_verify link unpolled, read by
  published seq ranges the GPU gathers, fd_verify_hip_tile_submit_range)
  gives the host copy's outcome counts at one and two tiles; with a
  producer under no flow control at all (TILE_RUN_NO_FLOW: the reference's
  unreliable link) on a shallow link, the tile is lapped, drops the lost
  frags as the stem drops an overrun, and keeps running.
- Two quic_verify links (as with two quic tiles; every verify tile reads
  every link): range mode (two range links, round robin) and the stem's
  polling (the first link GPU-copied, the second host-copied) at one and
  two tiles.  Arrival order across links differs between the two forms,
  so the counts compared are those the order cannot change: frags,
  signatures, parse failures, published, and published + dedup + verify
  failures.
The full-byte equality of the patched tile with the reference tile is
tests/test_gpu_tile_hip.py (mock topology, both copy forms via the kernel
tests in tests/test_gpu_txn_batch.py)."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))


@pytest.fixture(scope="module")
def stream(tmp_path_factory, verifier):
    import tile_bench as TB
    assert os.path.exists(os.path.join(TB.BUILD, "tile_run")), "integration/_build missing: run build()"
    p = str(tmp_path_factory.mktemp("tile_run") / "stream.bin")
    s = TB.make_stream(1 << 18, p, seed=0x7e60)
    return p, s


def _outcomes(r):
    return {k: r[k] for k in ("frags", "sigs", "published", "parse_fail", "verify_fail", "dedup", "bundle_peer_fail")}


def test_gpu_copy_equals_host_copy(stream, tmp_path):
    import tile_bench as TB
    path, s = stream
    g = TB.run_one(os.path.join(TB.BUILD, "tile_run"), path, 1, 262144, 120, str(tmp_path / "gpu"))
    h = TB.run_one(os.path.join(TB.BUILD, "tile_run_hostcopy"), path, 1, 262144, 120, str(tmp_path / "host"))
    assert g["gpu_copy"] == 1 and h["gpu_copy"] == 0
    assert g["overrun"] == 0 and h["overrun"] == 0
    assert _outcomes(g) == _outcomes(h)
    assert g["frags"] == s.n and g["published"] > 0.5 * s.n and g["dedup"] > 0


def test_overruns_are_dropped_not_fatal(stream, tmp_path, monkeypatch):
    import tile_bench as TB
    path, s = stream
    monkeypatch.setenv("TILE_RUN_NO_MARGIN", "1")
    r = TB.run_one(os.path.join(TB.BUILD, "tile_run"), path, 1, 16384, 120, str(tmp_path / "ovr"))
    assert r["overrun"] > 0, r
    assert r["frags"] + r["overrun"] == s.n


@pytest.mark.parametrize("tiles", [1, 2])
def test_range_mode_equals_host_copy(stream, tmp_path, tiles):
    import tile_bench as TB
    path, s = stream
    r = TB.run_one(os.path.join(TB.BUILD, "tile_run"), path, tiles, 131072, 120, str(tmp_path / "range"),
                   range_mode=True)
    h = TB.run_one(os.path.join(TB.BUILD, "tile_run_hostcopy"), path, tiles, 131072, 120, str(tmp_path / "host"))
    assert r["range"] == 1 and h["range"] == 0
    assert r["overrun"] == 0 and h["overrun"] == 0
    assert _outcomes(r) == _outcomes(h)
    assert r["frags"] == s.n


@pytest.mark.parametrize("tiles", [1, 2])
def test_range_mode_overrun_is_dropped(stream, tmp_path, monkeypatch, tiles):
    import tile_bench as TB
    path, s = stream
    monkeypatch.setenv("TILE_RUN_NO_FLOW", "1")
    r = TB.run_one(os.path.join(TB.BUILD, "tile_run"), path, tiles, 4096, 120, str(tmp_path / "rovr"),
                   range_mode=True)
    assert r["overrun"] > 0, r
    assert r["frags"] + r["overrun"] == s.n


@pytest.mark.parametrize("tiles", [1, 2])
def test_two_links_range_and_polled(stream, tmp_path, tiles):
    import tile_bench as TB
    path, s = stream
    exe = os.path.join(TB.BUILD, "tile_run")
    depth = 262144 * tiles                  # the polled tiles hold (INFLIGHT+1) x 2 x BATCH_MAX frags each
    r = TB.run_one(exe, path, tiles, depth, 120, str(tmp_path / "range"), range_mode=True, links=2)
    p = TB.run_one(exe, path, tiles, depth, 120, str(tmp_path / "polled"), links=2)
    assert r["links"] == 2 and p["links"] == 2 and r["range"] == 1 and p["range"] == 0
    assert r["overrun"] == 0 and p["overrun"] == 0
    for k in ("frags", "sigs", "parse_fail", "published"):
        assert r[k] == p[k], (k, r[k], p[k])
    assert r["frags"] == s.n
    assert r["published"] + r["dedup"] + r["verify_fail"] == p["published"] + p["dedup"] + p["verify_fail"]


@pytest.mark.parametrize("range_mode", [False, True])
@pytest.mark.parametrize("out_depth", [256, 16384])
def test_stalled_consumer_reads_the_reference_sequence(tmp_path, monkeypatch, range_mode, out_depth):
    """a reliable consumer of the out link (TILE_RUN_CONS: tile_run.c's
    drv_cons) that stalls 300 ms while a third of the frags are dropped
    (parse / verify / dedup): the tile's frags on the GPU and the dropped
    ones hold out chunks without credits, so only the chunk ring check
    (verify_hip_room) keeps the tile from overwriting a frag the consumer
    has not read.  The consumer's digest of every payload it reads, in
    order, equals the reference tile's over the same stream, at the
    reference's default out depth (16384) and a shallow one (256), with the
    reference's stem burst of 1."""
    import numpy as np
    import svc_io as S
    import tile_bench as TB
    import txn_lib as T
    from firedancer_amd.txn_workload import make_txn_stream
    from tile_io import read_fdo1, run_driver, write_fdt1
    s = make_txn_stream(3000, T.oracle_signer, seed=0x7e6a, dup_frac=0.15, graft_frac=0.02, bad_frac=0.2)
    p = str(tmp_path / "s.bin")
    write_fdt1(p, s.pool, s.off, s.sz, np.zeros(s.n, np.uint64), 0x5eed7117, 777)
    run_driver("ref", p, str(tmp_path / "ref.bin"))
    ref = S.reference_digest(read_fdo1(str(tmp_path / "ref.bin"), 777))
    monkeypatch.setenv("TILE_RUN_CONS", "1")
    monkeypatch.setenv("TILE_RUN_CONS_STALL_MS", "300")
    monkeypatch.setenv("TILE_RUN_OUT_DEPTH", str(out_depth))
    r = TB.run_one(os.path.join(TB.BUILD, "tile_run"), p, 1, 262144, 120, str(tmp_path / "run"), range_mode=range_mode)
    t = r["tiles"][0]
    assert r["overrun"] == 0 and t["cons_bad"] == 0, r
    assert t["consumed"] == t["published"] == ref["published"]
    assert int(t["cons_digest"], 16) == ref["digest"]
    assert (t["parse_fail"], t["verify_fail"], t["dedup"]) == (ref["parse_fail"], ref["verify_fail"], ref["dedup"])
