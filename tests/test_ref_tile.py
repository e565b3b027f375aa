"""CPU: the reference's own verify tile (src/disco/verify/fd_verify_tile.c,
compiled from its sources by oracle/Makefile) driven through its mock
topology (oracle/tile_drv.c, after test_verify_tile.c) over the committed C4
stream (tests/golden/c4_stream_2048.npz).

- With integration/fd_verify_tile_hip.patch and FD_HAS_HIP off (the reference
  tile plus the patch's tcache-footprint fix) it reproduces the fixture
  exactly: published frags, their bytes, metrics and the final tcache.
- The tile as it lies does not: fd_verify_tile.c:180 reserves
  FD_TCACHE_FOOTPRINT( depth, 0UL ), which omits the default map
  (fd_tcache.h:35-38), while fd_tcache_new( ..., 0UL ) lays one out
  (fd_tcache.c:11,27) -- the 12 fd_sha512_t scratch objects appended next
  (:186-190) overlap the map, and hashing overwrites map slots.  The test
  pins that diagnosis: its map holds values that are not tags in its ring,
  and it misses dedups the fixed tile catches.
- The GPU tile (FD_HAS_HIP) compiles and links against the engine; it runs
  in tests/test_gpu_tile_hip.py."""
import os
import subprocess

import numpy as np
import pytest

from tile_io import REF_DIR, check_against_stream, read_fdo1, run_driver, write_fdt1

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(REF_DIR, "tile_drv_ref")),
                                reason="tile drivers need /root/reference (built by build())")


@pytest.fixture(scope="module")
def c4(tmp_path_factory):
    d = dict(np.load(os.path.join(GOLDEN, "c4_stream_2048.npz")))
    p = str(tmp_path_factory.mktemp("tile") / "in.bin")
    write_fdt1(p, d["pool"], d["off"], d["sz"], d["bundle_id"], d["seed"], d["depth"])
    return d, p


def test_fixed_reference_tile_equals_fixture(c4, tmp_path):
    d, inp = c4
    out_p = str(tmp_path / "ref.bin")
    run_driver("ref", inp, out_p)
    out = read_fdo1(out_p, int(d["depth"]))
    check_against_stream(out, d["pool"], d["off"], d["sz"], d["result"], d["txn_t_sz"], d["metrics"])
    assert out["oldest"] == int(d["oldest"])
    assert np.array_equal(out["ring"], d["ring"]) and np.array_equal(out["map"], d["map"])
    live = set(int(t) for t in out["ring"] if t)
    assert set(int(t) for t in out["map"] if t) == live        # the map holds exactly the ring's tags


def test_reference_tile_as_is_has_overlapping_tcache(c4, tmp_path):
    d, inp = c4
    out_p = str(tmp_path / "orig.bin")
    run_driver("orig", inp, out_p)
    out = read_fdo1(out_p, int(d["depth"]))
    ring = set(int(t) for t in out["ring"] if t)
    stray = [int(t) for t in out["map"] if t and int(t) not in ring]
    assert stray, "expected map slots overwritten by the sha512 scratch"
    assert out["metrics"][2] < d["metrics"][2]              # dedups lost
    assert len(out["frags"]) > int((d["result"] == 0).sum())


def test_gpu_tile_links_against_engine():
    exe = os.path.join(REF_DIR, "tile_drv_hip")
    assert os.path.exists(exe)
    deps = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
    assert "libfd_ed25519_hip.so" in deps
    syms = subprocess.run(["nm", "-u", exe], capture_output=True, text=True).stdout
    for s in ("fd_verify_hip_tile_poll", "fd_verify_hip_tile_submit_frags", "fd_verify_hip_tile_complete",
              "fd_ed25519_hip_host_register"):
        assert s in syms, s
