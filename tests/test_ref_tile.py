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
  in tests/test_gpu_tile_hip.py.
- integration/fd_verify_topo_hip.patch applies to both of the reference's
  topologies and changes exactly one thing in each: the verify tiles'
  quic_verify in link is FD_TOPOB_UNPOLLED when FD_HAS_HIP (range mode,
  tests/test_gpu_tile_run.py), FD_TOPOB_POLLED otherwise."""
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


REF = "/root/reference"


def _strip_svc(lines):
    """the lines outside #if FD_HAS_HIP_SVC ... #endif blocks (the service
    mode's additions, checked separately)"""
    out, depth = [], 0
    for x in lines:
        if depth:
            depth += x.startswith("#if")
            depth -= x.startswith("#endif")
            continue
        if x.startswith("#if FD_HAS_HIP_SVC"):
            depth = 1
            continue
        out.append(x)
    return out


@pytest.mark.skipif(not os.path.isdir(REF), reason="needs /root/reference")
def test_topology_patch_applies_and_only_unpolls_quic_verify(tmp_path):
    """integration/fd_verify_topo_hip.patch: both topologies' quic_verify in
    links unpolled with FD_HAS_HIP or FD_HAS_HIP_SVC; everything else it
    adds sits in FD_HAS_HIP_SVC blocks (the GPU tiles, their verify_svc
    objects and registrations, the GPU tile's sandbox opt-out), and the
    patched files of both apps compile with FD_HAS_HIP_SVC against the
    reference's headers."""
    import shutil
    topos = ["src/app/fdctl/topology.c", "src/app/firedancer/topology.c"]
    others = ["src/app/fdctl/main.c", "src/app/firedancer/main.c", "src/disco/topo/fd_topo_run.c"]
    for f in topos + others:
        os.makedirs(tmp_path / os.path.dirname(f), exist_ok=True)
        shutil.copy(os.path.join(REF, f), tmp_path / f)
    patch = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "integration",
                         "fd_verify_topo_hip.patch")
    subprocess.check_call(["patch", "-s", "-p1", "-i", patch], cwd=tmp_path)
    for f in topos:
        old = open(os.path.join(REF, f)).read().splitlines()
        new = _strip_svc(open(tmp_path / f).read().splitlines())
        changed = [(a, b) for a, b in zip([x for x in old if "quic_verify" in x and "verify\"," in x],
                                          [x for x in new if "quic_verify" in x and "verify\"," in x])]
        tile_in = [(a, b) for a, b in changed if "fd_topob_tile_in" in a]
        assert len(tile_in) == 1 and tile_in[0][1] == tile_in[0][0].replace("FD_TOPOB_POLLED", "FD_VERIFY_QUIC_POLL")
        body = "\n".join(new)
        assert "#define FD_VERIFY_QUIC_POLL FD_TOPOB_UNPOLLED" in body and "#define FD_VERIFY_QUIC_POLL FD_TOPOB_POLLED" in body
        # every other line is the reference's
        extra = [x for x in new if x not in old]
        assert all("FD_VERIFY_QUIC_POLL" in x or x.startswith(("/*", "   ", "#if", "#else", "#endif")) or not x.strip()
                   for x in extra), extra
    for f in others:
        assert _strip_svc(open(tmp_path / f).read().splitlines()) == open(os.path.join(REF, f)).read().splitlines(), f
    # both topologies get the GPU tiles and their verify_svc objects, shaped by fd_verify_svc_topo_shape
    # (tests/test_svc_shape.py: every verify tile count boots), and both mains register them
    for f in topos:
        fd = open(tmp_path / f).read()
        assert '"vgpu"' in fd and "fd_verify_svc_tiles_on" in fd and "verify_svc.gpu_cnt" in fd, f
        assert "fd_verify_svc_topo_shape" in fd and "obj.%lu.slot_cap" in fd and "32768UL,  \"obj" not in fd, f
    for f in ["src/app/fdctl/main.c", "src/app/firedancer/main.c"]:
        fd = open(tmp_path / f).read()
        assert "&fd_obj_cb_verify_svc" in fd and "&fd_tile_verify_gpu" in fd, f
    for f in topos + others:
        subprocess.check_call(["gcc", "-std=c17", "-DFD_HAS_HOSTED=1", "-DFD_HAS_INT128=1", "-DFD_HAS_DOUBLE=1",
                               "-DFD_HAS_ALLOCA=1", "-DFD_HAS_X86=1", "-DFD_HAS_ATOMIC=1", "-DFD_HAS_THREADS=1",
                               "-DFD_HAS_HIP_SVC=1", "-fsyntax-only", "-Wall", "-Werror"] +
                              ([] if f.endswith("fd_topo_run.c") else ["-D_GNU_SOURCE"]) + [
                               "-I" + os.path.join(REF, os.path.dirname(f)),
                               "-I" + os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include"),
                               str(tmp_path / f)])


def test_gpu_tile_compiles_against_reference_headers():
    """integration/fd_verify_gpu_tile.c (the topology's vgpu tile and the
    verify_svc object callbacks) under -Wall -Wextra -Werror"""
    obj = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "integration", "_build",
                       "verify_gpu_tile.o")
    if not os.path.exists(obj):
        pytest.skip("integration/_build missing")
    syms = subprocess.run(["nm", obj], capture_output=True, text=True).stdout
    for s_ in ("fd_tile_verify_gpu", "fd_obj_cb_verify_svc", "fd_verify_svc_boot", "fd_verify_svc_poll"):
        assert s_ in syms, s_


def test_tile_run_uses_range_entry_points():
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "integration", "_build", "tile_run")
    if not os.path.exists(exe):
        pytest.skip("integration/_build missing")
    syms = subprocess.run(["nm", "-u", exe], capture_output=True, text=True).stdout
    for s_ in ("fd_verify_hip_tile_submit_range", "fd_verify_hip_tile_complete_range"):
        assert s_ in syms, s_


def test_patched_tile_compiles_warning_free():
    """integration/Makefile's tile_run_strict.o: the patched fd_verify_tile.c
    (both patches' tile side, range mode included) and tile_run.c under
    -Wall -Wextra -Werror (the populate_allowed_* hooks excepted: tile_run
    drives the callbacks itself)."""
    obj = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "integration", "_build",
                       "tile_run_strict.o")
    if not os.path.exists(obj):
        pytest.skip("integration/_build missing")
    syms = subprocess.run(["nm", obj], capture_output=True, text=True).stdout
    for s_ in ("fd_verify_hip_tile_submit_range", "fd_verify_hip_tile_complete_range",
               "fd_verify_hip_tile_set_staging", "fd_verify_hip_tile_submit_frags"):
        assert s_ in syms, s_                  # the range, staging and stem paths are compiled in


@pytest.mark.skipif(not os.path.isdir(REF), reason="needs /root/reference")
def test_metrics_patch_extends_the_verify_schema(tmp_path):
    """integration/fd_verify_metrics_hip.patch: the verify tile's GPU metrics
    in metrics.xml and in its generated header and table, laid out as
    gen_metrics.py lays them out (src/disco/metrics/generate/types.py: each
    counter one slot, each histogram FD_HISTF_BUCKET_CNT + 1 = 17 slots, after
    the tile's existing ones), inside the tile's metric area"""
    import re
    import shutil
    import xml.etree.ElementTree as ET
    files = ["src/disco/metrics/metrics.xml", "src/disco/metrics/generated/fd_metrics_verify.h",
             "src/disco/metrics/generated/fd_metrics_verify.c"]
    for f in files:
        os.makedirs(tmp_path / os.path.dirname(f), exist_ok=True)
        shutil.copy(os.path.join(REF, f), tmp_path / f)
    patch = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "integration",
                         "fd_verify_metrics_hip.patch")
    subprocess.check_call(["patch", "-s", "-p1", "-i", patch], cwd=tmp_path)
    root = ET.parse(tmp_path / files[0]).getroot()
    verify = [t for t in root.findall("tile") if t.attrib["name"] == "verify"][0]
    names = [m.attrib["name"] for m in verify]
    assert names[-4:] == ["GpuSignatures", "GpuHostRedone", "GpuIngestLatencyNanos", "GpuBatchLatencyNanos"]
    h = open(tmp_path / files[1]).read()
    off = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define FD_METRICS_\w+?_VERIFY_(\w+)_OFF\s+\((\d+)UL\)", h)}
    slots, at = {"counter": 1, "histogram": 17}, 16
    for m in verify:
        key = re.sub(r"(?<!^)(?=[A-Z])", "_", m.attrib["name"]).upper()
        assert off[key] == at, (key, off[key], at)
        at += slots[m.tag]
    all_h = open(os.path.join(REF, "src/disco/metrics/generated/fd_metrics_all.h")).read()
    total = 8 * 254
    assert f"#define FD_METRICS_TOTAL_SZ (8UL*254UL)" in all_h and 8 * at <= total
    assert "#define FD_METRICS_VERIFY_TOTAL (9UL)" in h
    c = open(tmp_path / files[2]).read()
    assert c.count("DECLARE_METRIC") == 9 and "DECLARE_METRIC_HISTOGRAM_NONE( VERIFY_GPU_BATCH_LATENCY_NANOS )" in c
