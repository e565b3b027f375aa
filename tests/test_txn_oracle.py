"""Verify-tile oracle (oracle/fd_txn_oracle.c) pinned against the reference's
own fixtures and its build from source, plus the engine's host-side pieces
(fd_hash, tcache) that run without a GPU.  CPU only."""
import json
import os

import numpy as np
import pytest

import txn_lib as T

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def tv():
    with open(os.path.join(GOLD, "txn_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def c4():
    return dict(np.load(os.path.join(GOLD, "c4_stream_2048.npz")))


def test_fd_hash_vectors(tv):
    from firedancer_amd import verify_tile as V
    for v in tv["fd_hash"]:
        b = bytes.fromhex(v["in"])
        seed = int(v["seed"])
        assert T.olib().oracle_fd_hash(seed, b, len(b)) == int(v["out"])
        assert V.fd_hash(seed, b) == int(v["out"])            # the engine's host entry


def test_parse_fixtures(tv):
    for p in tv["parse"]:
        n, out = T.oracle_parse(bytes.fromhex(p["payload"]))
        assert n == p["footprint"], p["name"]
        assert out.hex() == p["txn_t"], p["name"]


def _mutation_sweep(payload):
    """test_txn_parse.c:test_mutate: every truncation and every single-byte value."""
    L = len(payload)
    base = np.frombuffer(payload, np.uint8)
    pays = [base[:i] for i in range(L)]
    for i in range(L):
        for d in range(1, 256):
            q = base.copy(); q[i] = (int(q[i]) + d) & 0xff
            pays.append(q)
    sz = np.array([p.size for p in pays], np.uint16)
    off = np.zeros(len(pays), np.uint64); off[1:] = np.cumsum(sz.astype(np.uint64))[:-1]
    return np.concatenate(pays + [np.zeros(8, np.uint8)]), off.astype(np.uint32), sz


@pytest.mark.parametrize("k", [1, 2])
def test_parse_mutation_sweep_vs_reference(tv, k):
    if not T.have_ref():
        pytest.skip("reference build (oracle/_ref) not present")
    payload = bytes.fromhex(tv["parse"][k - 1]["payload"])
    pool, off, sz = _mutation_sweep(payload)
    tsz, out = T.oracle_parse_many(pool, off, sz)
    ok = 0
    for j in range(off.size):
        n, ref = T.ref_parse(pool[off[j]:off[j] + sz[j]].tobytes())
        assert tsz[j] == n, j
        if n:
            assert out[j, :n].tobytes() == ref, j
            ok += 1
    assert 0 < ok < off.size


def test_parse_stream_vs_reference(c4):
    if not T.have_ref():
        pytest.skip("reference build (oracle/_ref) not present")
    tsz, out = T.oracle_parse_many(c4["pool"], c4["off"], c4["sz"])
    assert np.array_equal(tsz, c4["txn_t_sz"])
    for j in range(0, c4["off"].size, 7):
        n, ref = T.ref_parse(c4["pool"][c4["off"][j]:c4["off"][j] + c4["sz"][j]].tobytes())
        assert n == tsz[j] and out[j, :n].tobytes() == ref


def _replay(tile, txns, seq, run_one):
    got, bid = [], 1000
    for step in seq:
        if step == "reset":
            tile.reset_tcache(); continue
        name, dedup, _ = step
        got.append(run_one(tile, np.frombuffer(bytes.fromhex(txns[name]), np.uint8), None if dedup else bid))
        bid += 1
    return got


def _oracle_one(tile, p, bid):
    res, _, _ = tile.run(p, np.zeros(1, np.uint32), np.array([p.size], np.uint16),
                         None if bid is None else np.array([bid], np.uint64))
    return int(res[0])


def test_verify_sequences(tv):
    """src/disco/verify/test_verify.c, every FD_TEST(res==...) in order."""
    for name, seq in tv["verify_seqs"].items():
        tile = T.OracleTile(seed=0x1234, depth=16, map_cnt=64)
        got = _replay(tile, tv["verify_txns"], seq, _oracle_one)
        assert got == [s[2] for s in seq if s != "reset"], name


def test_c4_stream_fixture(c4):
    tile = T.OracleTile(seed=int(c4["seed"]), depth=int(c4["depth"]))
    res, tag, tsz = tile.run(c4["pool"], c4["off"], c4["sz"], c4["bundle_id"])
    assert np.array_equal(res, c4["result"])
    assert np.array_equal(tag, c4["tag"])
    assert np.array_equal(tsz, c4["txn_t_sz"])
    m = tile.metrics()
    assert [m[k] for k in ("parse_fail_cnt", "verify_fail_cnt", "dedup_fail_cnt", "bundle_peer_fail_cnt")] == \
        c4["metrics"].tolist()
    assert np.array_equal(tile.ring, c4["ring"]) and np.array_equal(tile.map, c4["map"])
    assert tile.oldest == int(c4["oldest"])
    # every outcome class is present in the fixture
    assert set(np.unique(res).tolist()) == {0, -1, -2, -3, -4}


def test_c4_stream_split_batches_vs_reference(c4):
    """Feeding the stream in several calls keeps tcache + bundle state."""
    if not T.have_ref():
        pytest.skip("reference build (oracle/_ref) not present")
    o = T.OracleTile(seed=99, depth=64)
    r = T.RefTile(seed=99, depth=64)
    cuts = [0, 1, 300, 301, 1024, 2048]
    for a, b in zip(cuts[:-1], cuts[1:]):
        ro = o.run(c4["pool"], c4["off"][a:b], c4["sz"][a:b], c4["bundle_id"][a:b])
        rr = r.run(c4["pool"], c4["off"][a:b], c4["sz"][a:b], c4["bundle_id"][a:b])
        for x, y in zip(ro, rr):
            assert np.array_equal(x, y)
    assert o.metrics() == r.metrics()
    assert np.array_equal(o.ring, r.ring) and np.array_equal(o.map, r.map) and o.oldest == r.oldest


def test_engine_tcache_matches_oracle():
    """The engine's host tcache (fd_verify_hip_tcache_*) against the oracle's
    restatement on a random insert/query stream with heavy eviction."""
    from firedancer_amd import verify_tile as V
    rng = np.random.default_rng(3)
    depth, map_cnt = 37, 128
    tc = V.Tcache(depth, map_cnt)
    ring = np.zeros(depth, np.uint64); mp = np.zeros(map_cnt, np.uint64); oldest = np.zeros(1, np.uint64)
    L = T.olib()
    # tags that collide in the low bits, so probe chains and backward shifts are exercised
    tags = (rng.integers(1, 400, 6000).astype(np.uint64) * np.uint64(map_cnt // 4) + rng.integers(0, 3, 6000)
            .astype(np.uint64))
    for t in tags:
        t = int(t)
        if rng.random() < 0.3:
            assert tc.query(t) == bool(L.oracle_tcache_query(mp.ctypes.data, map_cnt, t))
        else:
            a = tc.insert(t)
            b = bool(L.oracle_tcache_insert(oldest.ctypes.data, ring.ctypes.data, depth, mp.ctypes.data, map_cnt, t))
            assert a == b
            assert np.array_equal(tc.map, mp) and np.array_equal(tc.ring, ring) and tc.oldest[0] == oldest[0]
    assert tc.query(0)          # the null tag always "finds"
    assert V.lib().fd_verify_hip_tcache_map_cnt_default(4194302) == L.oracle_tcache_map_cnt_default(4194302) == 1 << 23


def test_generator_shapes():
    from firedancer_amd.txn_workload import make_txn_stream
    s = make_txn_stream(4000, T.oracle_signer, seed=11, mix="c1", dup_frac=0, graft_frac=0, bad_frac=0)
    tsz, _ = T.oracle_parse_many(s.pool, s.off, s.sz, want_out=False)
    assert (tsz > 0).all()                                 # every generated txn parses
    assert s.sz.max() <= 1232 and s.nsig.max() <= 12 and s.nsig.min() >= 1
    frac1 = (s.nsig == 1).mean()
    assert 0.76 < frac1 < 0.84
    tile = T.OracleTile(seed=5, depth=1 << 14)
    res, _, _ = tile.run(s.pool, s.off, s.sz)
    assert (res == 0).all()                                # all valid, no dups: everything publishes
