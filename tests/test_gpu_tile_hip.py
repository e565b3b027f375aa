"""GPU: the reference verify tile patched for the engine
(integration/fd_verify_tile_hip.patch, FD_HAS_HIP) against the reference
tile itself, both driven through the reference's mock topology
(oracle/tile_drv.c after src/disco/verify/test_verify_tile.c; stem callback
order of src/disco/stem/fd_stem.c:506-712).

The patched tile keeps during_frag's copy into the out dcache, queues frags
in after_frag, sends full batches to the GPU (parse in place in the
registered out dcache, verify, per-txn reduce), and from after_credit polls
the oldest batch without blocking (fd_verify_hip_tile_poll), runs the
ordered tcache / bundle pass and publishes in arrival order.  The reference
tile (tile_drv_ref: the same patch with FD_HAS_HIP off, i.e. the reference
plus its tcache-footprint fix, tests/test_ref_tile.py) runs the same stream
on the host CPU.  The driver outputs -- every published frag's mcache
fields and dcache bytes (header, payload, fd_txn_t), the metrics and the
final tcache -- must be byte-identical (apart from the one alignment pad
byte before an odd payload's fd_txn_t, which the reference never writes).  The committed C4 fixture is also
checked directly, so the comparison does not rest on the reference binary
alone.  One run enters the patched tile's seccomp policy before the first
frag (syscalls outside it trap and are counted) and must see none."""
import os

import numpy as np
import pytest

import txn_lib as T
from tile_io import check_against_stream, normalized, read_fdo1, run_driver, write_fdt1

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _c4(tmp_path):
    d = dict(np.load(os.path.join(GOLDEN, "c4_stream_2048.npz")))
    p = str(tmp_path / "c4.bin")
    write_fdt1(p, d["pool"], d["off"], d["sz"], d["bundle_id"], d["seed"], d["depth"])
    return d, p


def test_patched_tile_equals_reference_tile_c4(tmp_path):
    d, inp = _c4(tmp_path)
    run_driver("ref", inp, str(tmp_path / "ref.bin"))
    log = run_driver("hip", inp, str(tmp_path / "hip.bin"))
    ref = read_fdo1(str(tmp_path / "ref.bin"), int(d["depth"]))
    hip = read_fdo1(str(tmp_path / "hip.bin"), int(d["depth"]))
    check_against_stream(hip, d["pool"], d["off"], d["sz"], d["result"], d["txn_t_sz"], d["metrics"])
    assert hip["oldest"] == int(d["oldest"]) and np.array_equal(hip["ring"], d["ring"])
    assert np.array_equal(hip["map"], d["map"])
    assert normalized(hip) == normalized(ref)
    assert "published 1420 of 2048" in log


def test_patched_tile_under_its_seccomp_policy(tmp_path):
    d, inp = _c4(tmp_path)
    log = run_driver("hip", inp, str(tmp_path / "hip.bin"), env={"TILE_DRV_SECCOMP": "1"})
    assert "seccomp traps: 0" in log, [l for l in log.splitlines() if "seccomp" in l]
    hip = read_fdo1(str(tmp_path / "hip.bin"), int(d["depth"]))
    check_against_stream(hip, d["pool"], d["off"], d["sz"], d["result"], d["txn_t_sz"], d["metrics"])


def test_patched_tile_equals_reference_tile_generated_stream(tmp_path):
    """12 000 generated frags (resends, grafted sig0, malformed frags,
    bundles): 12 GPU batches, two in flight, the blocking submit when both
    slots are taken, and the partial-batch flush at the end."""
    from firedancer_amd.txn_workload import make_txn_stream
    s = make_txn_stream(12000, T.oracle_signer, seed=0x7113, dup_frac=0.05, graft_frac=0.01, bad_frac=0.02)
    bid = np.zeros(s.n, np.uint64)
    r = np.random.default_rng(0x7114)
    for start in r.choice(s.n - 8, 100, replace=False):
        bid[start:start + int(r.integers(1, 6))] = int(r.integers(1, 2**40))
    inp = str(tmp_path / "gen.bin")
    depth = 777
    write_fdt1(inp, s.pool, s.off, s.sz, bid, 0x5eed7113, depth)
    run_driver("ref", inp, str(tmp_path / "ref.bin"))
    run_driver("hip", inp, str(tmp_path / "hip.bin"))
    ref = read_fdo1(str(tmp_path / "ref.bin"), depth)
    hip = read_fdo1(str(tmp_path / "hip.bin"), depth)
    assert len(hip["frags"]) == len(ref["frags"]) > 6000
    assert [t for _, t, _ in hip["frags"]] == [t for _, t, _ in ref["frags"]]
    assert np.array_equal(hip["metrics"], ref["metrics"])
    assert normalized(hip) == normalized(ref)
    assert ref["metrics"][2] > 100 and ref["metrics"][3] > 0     # dedups and bundle peers occurred


def test_range_mode_equals_reference_tile(tmp_path):
    """The quic link unpolled (range mode): the driver only publishes, the
    tile reads published seq ranges from after_credit and the GPU gathers the
    mcache lines; outputs byte-identical to the reference tile, on the C4
    fixture and the generated stream with bundles."""
    d, inp = _c4(tmp_path)
    run_driver("ref", inp, str(tmp_path / "ref.bin"))
    log = run_driver("hip", inp, str(tmp_path / "rng.bin"), env={"TILE_DRV_RANGE": "1"})
    ref = read_fdo1(str(tmp_path / "ref.bin"), int(d["depth"]))
    rng = read_fdo1(str(tmp_path / "rng.bin"), int(d["depth"]))
    check_against_stream(rng, d["pool"], d["off"], d["sz"], d["result"], d["txn_t_sz"], d["metrics"])
    assert normalized(rng) == normalized(ref)
    assert "published 1420 of 2048" in log
    from firedancer_amd.txn_workload import make_txn_stream
    s = make_txn_stream(12000, T.oracle_signer, seed=0x7115, dup_frac=0.05, graft_frac=0.01, bad_frac=0.02)
    bid = np.zeros(s.n, np.uint64)
    r = np.random.default_rng(0x7116)
    for start in r.choice(s.n - 8, 100, replace=False):
        bid[start:start + int(r.integers(1, 6))] = int(r.integers(1, 2**40))
    gen = str(tmp_path / "gen.bin")
    write_fdt1(gen, s.pool, s.off, s.sz, bid, 0x5eed7115, 777)
    run_driver("ref", gen, str(tmp_path / "gref.bin"))
    run_driver("hip", gen, str(tmp_path / "grng.bin"), env={"TILE_DRV_RANGE": "1"})
    a = read_fdo1(str(tmp_path / "gref.bin"), 777)
    b = read_fdo1(str(tmp_path / "grng.bin"), 777)
    assert len(b["frags"]) == len(a["frags"]) > 6000
    assert normalized(b) == normalized(a)
