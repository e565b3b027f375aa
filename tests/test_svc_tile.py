"""CPU: the service-mode verify tile (src/disco/verify/fd_verify_tile.c +
integration/fd_verify_tile_svc.patch, FD_HAS_HIP_SVC) in the reference's own
run loop (integration/svc_tile_run.c: a producer, the tiles in stem_run1,
one reliable verify_dedup consumer per tile), with oracle/_ref/svc_mock
standing in for the GPU tile: the same segment protocol
(include/fd_verify_svc.h) answered with the reference's own CPU parse and
verify.  These check the tile side of the protocol -- the ordered pass,
out chunks on publish only, flushes within the credits, publish order, the
overrun checks, the link metrics -- here, without a GPU; the same runs
against the GPU tile are tests/test_gpu_svc_run.py.

- One tile: the published payloads (in order, as a digest), the outcome
  counts and the tcache effects equal the reference tile's
  (oracle/tile_drv.c tile_drv_ref) on a generated stream with resends,
  grafted signatures, malformed payloads and bundles -- range mode and the
  stem-polled form.
- Two tiles: each tile's published sequence equals the reference tile run
  over that tile's round robin share.
- A consumer that stalls 300-500 ms behind a verify_dedup link of 128-256
  frags (the out dcache sized by the reference's rule for that depth,
  burst 1) and a stream where a third of the frags are dropped: every
  frag the consumer reads is intact and the sequence is still the
  reference's.  (chunks taken per frag, published or not,
  let a lagging consumer's unread frags be overwritten.)
- Each tile process has one thread and no /dev/kfd or /dev/dri fd after
  privileged_init (unshare( CLONE_NEWUSER )'s preconditions, fd_sandbox.c:640-655).
- The range links' counts land in the link-in metric slots after the
  polled links' (metrics_write)."""
import os
import subprocess

import numpy as np
import pytest

import svc_io as S
import txn_lib as T
from tile_io import read_fdo1, run_driver, write_fdt1

pytestmark = pytest.mark.skipif(not (os.path.exists(S.MOCK) and os.path.exists(os.path.join(S.BUILD, "svc_tile_run"))),
                                reason="svc_mock / svc_tile_run not built (build() with /root/reference)")

SEED, DEPTH = 0x5eed7117, 777
SMALL = {"SVC_RUN_SLOT_CAP": "1024", "SVC_RUN_REQ_DEPTH": "8"}


@pytest.fixture(scope="module")
def stream(tmp_path_factory):
    from firedancer_amd.txn_workload import make_txn_stream
    s = make_txn_stream(3000, T.oracle_signer, seed=0x7e62, dup_frac=0.05, graft_frac=0.01, bad_frac=0.02)
    bid = np.zeros(s.n, np.uint64)
    r = np.random.default_rng(0x7e63)
    for start in r.choice(s.n - 8, 40, replace=False):
        bid[start:start + int(r.integers(1, 6))] = int(r.integers(1, 2**40))
    d = tmp_path_factory.mktemp("svc")
    p = str(d / "stream.bin")
    write_fdt1(p, s.pool, s.off, s.sz, bid, SEED, DEPTH)
    run_driver("ref", p, str(d / "ref.bin"))
    ref = S.reference_digest(read_fdo1(str(d / "ref.bin"), DEPTH))
    return dict(path=p, s=s, bid=bid, ref=ref, dir=d)


def _check_run(r, n):
    assert r["overrun"] == 0 and r["lapped"] == 0 and r["consumer_bad"] == 0
    assert r["frags"] == n and r["consumed"] == r["published"]
    assert r["tile_threads_max"] == 1 and r["tile_dev_fds"] == 0


@pytest.mark.parametrize("polled", [0, 1])
def test_one_tile_equals_reference_tile(stream, tmp_path, polled):
    env = dict(SMALL)
    if polled:
        env.update(SVC_RUN_POLLED="1", SVC_RUN_FRAG_CAP="512")
    r = S.run(stream["path"], 1, 1 << 14, str(tmp_path / "run"), env=env, mock=True)
    _check_run(r, stream["s"].n)
    assert S.tile_counts(r["tiles"][0]) == stream["ref"]
    assert stream["ref"]["dedup"] > 50 and stream["ref"]["bundle_peer_fail"] > 0


def test_two_tiles_equal_reference_shares(stream, tmp_path):
    r = S.run(stream["path"], 2, 1 << 14, str(tmp_path / "run"), env=SMALL, mock=True)
    _check_run(r, stream["s"].n)
    for t in range(2):
        p = str(tmp_path / f"share{t}.bin")
        S.share_stream(p, stream["s"], stream["bid"], t, 2, SEED, DEPTH)
        run_driver("ref", p, str(tmp_path / f"ref{t}.bin"))
        assert S.tile_counts(r["tiles"][t]) == S.reference_digest(read_fdo1(str(tmp_path / f"ref{t}.bin"), DEPTH)), t


def test_credits_return_at_ingest(stream, tmp_path):
    """the stand-in answers in two steps as the GPU tile does (ingest ->
    INGESTED, verify 2 ms later -> RESULTS): each tile moves its link fseq at
    INGESTED, before the results (early_credits counts those ranges), and the
    published sequences are still the reference's; answering in one step,
    no range returns its credits early"""
    r = S.run(stream["path"], 2, 1 << 14, str(tmp_path / "run"), env=dict(SMALL, SVC_MOCK_INGEST="2000"), mock=True)
    _check_run(r, stream["s"].n)
    assert all(x["early_credits"] > 0 for x in r["tiles"])
    for t in range(2):
        p = str(tmp_path / f"share{t}.bin")
        S.share_stream(p, stream["s"], stream["bid"], t, 2, SEED, DEPTH)
        run_driver("ref", p, str(tmp_path / f"ref{t}.bin"))
        assert S.tile_counts(r["tiles"][t]) == S.reference_digest(read_fdo1(str(tmp_path / f"ref{t}.bin"), DEPTH)), t
    r1 = S.run(stream["path"], 2, 1 << 14, str(tmp_path / "run1"), env=SMALL, mock=True)
    assert all(x["early_credits"] == 0 for x in r1["tiles"])


def test_stalled_consumer_and_drops(tmp_path):
    """a third of the frags dropped (bad payloads, resends), the consumer
    stalled behind a 128-frag verify_dedup link: nothing overwritten"""
    from firedancer_amd.txn_workload import make_txn_stream
    s = make_txn_stream(2000, T.oracle_signer, seed=0x7e64, dup_frac=0.15, graft_frac=0.02, bad_frac=0.2)
    p = str(tmp_path / "s.bin")
    write_fdt1(p, s.pool, s.off, s.sz, np.zeros(s.n, np.uint64), SEED, DEPTH)
    run_driver("ref", p, str(tmp_path / "ref.bin"))
    ref = S.reference_digest(read_fdo1(str(tmp_path / "ref.bin"), DEPTH))
    assert ref["published"] < 0.7 * s.n
    env = dict(SMALL, SVC_RUN_CONS_STALL_MS="400", SVC_RUN_OUT_DEPTH="128")
    r = S.run(p, 1, 1 << 14, str(tmp_path / "run"), env=env, mock=True)
    _check_run(r, s.n)
    assert S.tile_counts(r["tiles"][0]) == ref
    assert r["regime"]["backpressure"] > 0.1                 # the tile waited for credits


def test_link_metrics_written(stream, tmp_path):
    r = S.run(stream["path"], 2, 1 << 14, str(tmp_path / "run"), env=SMALL, mock=True)
    assert r["metrics_ok"] == 1
    for t, x in enumerate(r["tiles"]):
        share = len(range(t, stream["s"].n, 2))
        assert x["link"]["consumed"] == share
        assert x["link"]["consumed"] + x["link"]["filtered"] == stream["s"].n
        assert x["link"]["overrun_polling"] == 0 and x["link"]["overrun_reading"] == 0
        # the GPU service's metrics in the verify tile's schema (integration/fd_verify_metrics_hip.patch:
        # metrics.xml's GpuSignatures, GpuHostRedone, GpuIngestLatencyNanos, GpuBatchLatencyNanos), written by
        # metrics_write: the counters equal the tile's own, each request with frags is one sample of each
        # histogram, and a request's results come after its ingest
        m = x["gpu_metrics"]
        assert m["signatures"] == x["sigs"] > 0 and m["host_redone"] == 0
        assert m["ingest_n"] == m["batch_n"] > 0 and 0 < m["ingest_mean_us"] <= m["batch_mean_us"]


def test_tile_to_gpu_assignment(tmp_path):
    """fd_verify_svc_gpu_of / _slot_of / _tiles_on:
    every verify tile on exactly one GPU's segment, slots dense per GPU"""
    src = tmp_path / "a.c"
    src.write_text('#include <stdio.h>\n#include "fd_verify_svc.h"\nint main(void){for(ulong g=1;g<=8;g++)'
                   'for(ulong v=1;v<=32;v++){for(ulong k=0;k<v;k++)printf("%lu %lu %lu %lu %lu\\n",g,v,k,'
                   'fd_verify_svc_gpu_of(k,g),fd_verify_svc_slot_of(k,g));for(ulong x=0;x<g;x++)'
                   'printf("T %lu %lu %lu %lu\\n",g,v,x,fd_verify_svc_tiles_on(x,v,g));}return 0;}\n')
    exe = tmp_path / "a"
    subprocess.check_call(["gcc", "-O1", "-Wall", "-Werror", "-I" + os.path.join(S.REPO, "include"), str(src), "-o", str(exe)])
    out = subprocess.check_output([str(exe)], text=True).split("\n")
    slots, on = {}, {}
    for line in out:
        f = line.split()
        if not f:
            continue
        if f[0] == "T":
            on[tuple(map(int, f[1:4]))] = int(f[4])
        else:
            g, v, k, gpu, slot = map(int, f)
            assert gpu < g
            slots.setdefault((g, v, gpu), []).append(slot)
    for (g, v, gpu), ss in slots.items():
        assert sorted(ss) == list(range(len(ss))), (g, v, gpu)        # dense, disjoint
        assert on[(g, v, gpu)] == len(ss)
    for g in range(1, 9):
        for v in range(1, 33):
            assert sum(on[(g, v, x)] for x in range(g)) == v


def test_svc_patch_compiles_strict():
    """the patched tile and svc_tile_run.c under -Wall -Wextra -Werror
    (integration/Makefile svc_tile_strict.o)"""
    assert os.path.exists(os.path.join(S.BUILD, "svc_tile_strict.o"))


def test_tiles_run_inside_the_reference_sandbox(stream, tmp_path):
    """SVC_RUN_SANDBOX=1: each tile enters the reference's fd_sandbox_enter
    after privileged_init (src/disco/topo/fd_topo_run.c:86-135) with its own
    populate_allowed_fds / populate_allowed_seccomp -- the reference's
    verify policy (write and fsync only), a user namespace, pivot_root,
    landlock, rlimits -- and still gives the reference's sequence.  Skipped
    where the container refuses user namespaces."""
    if subprocess.run(["unshare", "-U", "true"], capture_output=True).returncode:
        pytest.skip("user namespaces refused here")
    r = S.run(stream["path"], 2, 1 << 14, str(tmp_path / "run"), env=dict(SMALL, SVC_RUN_SANDBOX="1"), mock=True)
    _check_run(r, stream["s"].n)
    assert all(x["sandboxed"] == 1 for x in r["tiles"])
    for t in range(2):
        p = str(tmp_path / f"share{t}.bin")
        S.share_stream(p, stream["s"], stream["bid"], t, 2, SEED, DEPTH)
        run_driver("ref", p, str(tmp_path / f"ref{t}.bin"))
        assert S.tile_counts(r["tiles"][t]) == S.reference_digest(read_fdo1(str(tmp_path / f"ref{t}.bin"), DEPTH)), t


def _order_free(x):
    """counts no arrival order between links can change (a resend and its
    original on different links: which one publishes, and whether the other
    is a dedup or -- a grafted sig0 -- a verify failure, depends on the
    order; how many publish, and the sum, do not)"""
    return (x["published"], x["parse_fail"], x["published"] + x["dedup"] + x["verify_fail"])


@pytest.mark.parametrize("tiles", [1, 2])
def test_range_link_beside_a_polled_link(stream, tmp_path, tiles):
    """two quic_verify links on every tile, link 0 unpolled (range requests)
    and link 1 polled by the stem (frag requests through the frag area):
    per tile the order-free counts equal the reference's over the tile's
    share (seq % T of both links), and the all-range run's"""
    s = stream["s"]
    # no bundles (a bundle's frags split over two links are order-bound), and a
    # tcache that holds the whole stream (with 777 entries whether a resend is
    # caught depends on how far apart the two links put it and its original)
    p = str(tmp_path / "nobundle.bin")
    write_fdt1(p, s.pool, s.off, s.sz, np.zeros(s.n, np.uint64), SEED, 1 << 14)
    env = dict(SMALL, SVC_RUN_LINKS="2", SVC_RUN_FRAG_CAP="512")
    mixed = S.run(p, tiles, 1 << 14, str(tmp_path / "mixed"), env=dict(env, SVC_RUN_POLLED="2"), mock=True)
    rng = S.run(p, tiles, 1 << 14, str(tmp_path / "range"), env=env, mock=True)
    _check_run(mixed, s.n)
    _check_run(rng, s.n)
    for t in range(tiles):
        idx = np.array([j for j in range(s.n) if (j // 2) % tiles == t])   # frag j: link j % 2, seq j // 2
        ref = S.ref_share_digests(s.pool, s.off[idx], s.sz[idx], None, 1, SEED + t, 1 << 14)[0]
        assert _order_free(mixed["tiles"][t]) == _order_free(ref) == _order_free(rng["tiles"][t]), t
        assert mixed["tiles"][t]["sigs"] == rng["tiles"][t]["sigs"]
        assert mixed["tiles"][t]["link"]["consumed"] == len(range(t, (s.n + 1) // 2, tiles))   # the range link's share


def test_frags_shorter_than_their_payload_are_redone_on_the_tile(stream, tmp_path):
    """every 97th frag's mcache sz 8 bytes short of 80 + payload_sz
    (SVC_RUN_LIE): after_frag would parse 8 stale out-dcache bytes, so the
    tile redoes those frags as the reference tile does (FD_VERIFY_SVC_RES_HOST:
    its own copy, parse and CPU verify, published in order between the GPU's
    frags); every frag is accounted for, nothing read is torn, and the tile
    does not stall on its credits (a 256-frag out link)"""
    env = dict(SMALL, SVC_RUN_LIE="97", SVC_RUN_OUT_DEPTH="256")
    r = S.run(stream["path"], 1, 1 << 14, str(tmp_path / "run"), env=env, mock=True)
    _check_run(r, stream["s"].n)
    assert r["host_redone"] == len(range(96, stream["s"].n, 97))
    assert r["tiles"][0]["gpu_metrics"]["host_redone"] == r["host_redone"] and r["metrics_ok"] == 1



def test_lapped_polled_link_ends_the_run(tmp_path):
    """an unreliable producer far ahead of a shallow polled link: the stem
    skips the lapped frags itself (its link-in metrics count them, every
    tile's share alike), so a tile cannot count its share to the end -- it
    ends once the stem has passed the link's last seq, and the frags no tile
    saw are reported as unseen (the bench's lost count).  Before round 6 such
    a tile waited for its deadline: the paced polled bench runs timed out."""
    from firedancer_amd.txn_workload import make_txn_stream
    s = make_txn_stream(20000, T.oracle_signer, seed=0x7e6a)
    p = str(tmp_path / "s.bin")
    write_fdt1(p, s.pool, s.off, s.sz, np.zeros(s.n, np.uint64), SEED, DEPTH)
    r = S.run(p, 2, 256, str(tmp_path / "run"), mock=True, timeout=120,
              env={"SVC_RUN_POLLED": "1", "SVC_RUN_RATE": "50000000", "SVC_RUN_REQ_DEPTH": "16", "SVC_RUN_SLOT_CAP": "1024"})
    assert r["unseen"] > 0 and r["frags"] + r["overrun"] + r["lapped"] + r["unseen"] == s.n, r
    assert r["consumer_bad"] == 0 and r["consumed"] == r["published"]
