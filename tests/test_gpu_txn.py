"""GPU parity of the verify-tile layer (include/fd_verify_hip.h) against the
oracle restatement and the reference's fixtures: GPU fd_txn_parse (footprint
and fd_txn_t bytes), sig0 tags, and whole after_frag streams (per-frag result,
published tag, metrics, final tcache arrays).  Bit-exact everywhere."""
import json
import os

import numpy as np
import pytest

import txn_lib as T

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _dev(a, dtype_view=None):
    import torch
    a = np.ascontiguousarray(a)
    if dtype_view is not None:
        a = a.view(dtype_view)
    if a.size == 0:
        a = np.zeros(1, a.dtype)
    return torch.from_numpy(a).to("cuda:0")


def _frags(pool, off, sz):
    return _dev(pool), _dev(off.astype(np.uint32), np.int32), _dev(sz.astype(np.uint16), np.int16)


@pytest.fixture(scope="module")
def tv():
    with open(os.path.join(GOLD, "txn_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def c4():
    return dict(np.load(os.path.join(GOLD, "c4_stream_2048.npz")))


def gpu_parse(verifier, pool, off, sz):
    import torch
    from firedancer_amd import verify_tile as V
    n = off.size
    d_pool, d_off, d_sz = _frags(pool, off, sz)
    d_out = torch.zeros((max(n, 1), 852), dtype=torch.uint8, device="cuda:0")
    d_tsz = torch.zeros(max(n, 1), dtype=torch.int16, device="cuda:0")
    V.parse_dev(verifier, n, d_pool, d_off, d_sz, d_out, d_tsz)
    verifier.sync()
    return d_tsz.cpu().numpy().view(np.uint16)[:n], d_out.cpu().numpy()[:n]


def test_parse_fixtures(verifier, tv):
    for p in tv["parse"]:
        b = np.frombuffer(bytes.fromhex(p["payload"]), np.uint8)
        pool = np.concatenate([b, np.zeros(8, np.uint8)])
        tsz, out = gpu_parse(verifier, pool, np.zeros(1, np.uint32), np.array([b.size], np.uint16))
        assert int(tsz[0]) == p["footprint"], p["name"]
        assert out[0, :tsz[0]].tobytes().hex() == p["txn_t"], p["name"]


@pytest.mark.parametrize("k", [1, 2])
def test_parse_mutation_sweep(verifier, tv, k):
    """test_txn_parse.c:test_mutate's sweep (every truncation, every byte value)
    on the GPU, against the oracle (itself pinned to the reference build)."""
    from test_txn_oracle import _mutation_sweep
    pool, off, sz = _mutation_sweep(bytes.fromhex(tv["parse"][k - 1]["payload"]))
    tsz, out = gpu_parse(verifier, pool, off, sz)
    etsz, eout = T.oracle_parse_many(pool, off, sz)
    assert np.array_equal(tsz, etsz)
    ok = np.nonzero(etsz)[0]
    assert ok.size > 0
    for j in ok:
        n = etsz[j]
        assert np.array_equal(out[j, :n], eout[j, :n]), j


def test_parse_edge_cases(verifier):
    base = np.frombuffer(bytes.fromhex(json.load(open(os.path.join(GOLD, "txn_vectors.json")))["parse"][3]["payload"]),
                         np.uint8)
    pool = np.concatenate([base, np.zeros(2000, np.uint8)])
    off = np.array([0, 0, pool.size - 8, 0, 0], np.uint32)
    sz = np.array([base.size, 0, 0, 1233, 1232], np.uint16)     # ok, empty, empty at the end, > MTU, trailing zeros
    tsz, _ = gpu_parse(verifier, pool, off, sz)
    etsz, _ = T.oracle_parse_many(pool, off, sz)
    assert np.array_equal(tsz, etsz)
    assert tsz[0] == 20 and (tsz[1:] == 0).all()
    tsz, _ = gpu_parse(verifier, pool, off[:0], sz[:0])         # n = 0
    assert tsz.size == 0


def _tile(verifier, seed, depth, map_cnt=0, max_txn=4096):
    from firedancer_amd.verify_tile import VerifyTile
    return VerifyTile(verifier, max_txn=max_txn, hashmap_seed=seed, tcache_depth=depth, tcache_map_cnt=map_cnt)


def test_verify_sequences(verifier, tv):
    """src/disco/verify/test_verify.c through the GPU tile, one frag per batch."""
    for name, seq in tv["verify_seqs"].items():
        tile = _tile(verifier, 0x1234, 16, 64, max_txn=4)
        got, bid = [], 1000
        for step in seq:
            if step == "reset":
                tile.tcache_reset(); continue
            txn, dedup, _ = step
            p = np.frombuffer(bytes.fromhex(tv["verify_txns"][txn]), np.uint8)
            d = _frags(np.concatenate([p, np.zeros(8, np.uint8)]), np.zeros(1, np.uint32), np.array([p.size]))
            res, _, _ = tile.after_frags(1, *d, bundle_id=None if dedup else np.array([bid], np.uint64))
            bid += 1
            got.append(int(res[0]))
        tile.close()
        assert got == [s[2] for s in seq if s != "reset"], name


def test_c4_fixture_stream(verifier, c4):
    """The 2048-frag fixture (reference per-frag results, bundles, resends,
    grafted sig0, malformed frags) in one batch, with the tile joined to an
    external tcache so the final ring/map can be compared with the reference's."""
    from firedancer_amd.verify_tile import Tcache
    tile = _tile(verifier, int(c4["seed"]), int(c4["depth"]))
    tc = Tcache(int(c4["depth"]))
    tile.join_tcache(tc)
    d = _frags(c4["pool"], c4["off"], c4["sz"])
    res, tag, tsz = tile.after_frags(c4["off"].size, *d, bundle_id=c4["bundle_id"])
    assert np.array_equal(res, c4["result"])
    assert np.array_equal(tag, c4["tag"])
    assert np.array_equal(tsz, c4["txn_t_sz"])
    m = tile.metrics()
    assert [m[k] for k in ("parse_fail_cnt", "verify_fail_cnt", "dedup_fail_cnt", "bundle_peer_fail_cnt")] == \
        c4["metrics"].tolist()
    assert np.array_equal(tc.ring, c4["ring"]) and np.array_equal(tc.map, c4["map"])
    assert int(tc.oldest[0]) == int(c4["oldest"])
    tile.close()


def test_pipelined_batches_vs_oracle(verifier):
    """A 12000-frag generated stream in ragged batches, submitted one ahead
    (submit(k+1) before complete(k)), against the oracle over the whole stream;
    small tcache so eviction happens across batch boundaries."""
    from firedancer_amd.txn_workload import make_txn_stream
    s = make_txn_stream(12000, T.oracle_signer, seed=0xbeef, dup_frac=0.05, graft_frac=0.01, bad_frac=0.01)
    bid = np.zeros(s.n, np.uint64)
    r = np.random.default_rng(9)
    for start in r.choice(s.n - 8, 100, replace=False):
        bid[start:start + int(r.integers(1, 6))] = int(r.integers(1, 2**40))
    o = T.OracleTile(seed=77, depth=300)
    eres, etag, etsz = o.run(s.pool, s.off, s.sz, bid)
    tile = _tile(verifier, 77, 300, max_txn=4096)
    d_pool = _dev(s.pool)
    cuts = [0, 1, 64, 65, 4096 + 65, 6000, 6001, 9999, 12000]
    batches = list(zip(cuts[:-1], cuts[1:]))
    keep = []

    def submit(a, b):
        d_off, d_sz = _dev(s.off[a:b], np.int32), _dev(s.sz[a:b], np.int16)
        keep.append((d_off, d_sz))
        tile.submit(b - a, d_pool, d_off, d_sz)

    got, gpu_ms = [], []
    submit(*batches[0])
    for k, (a, b) in enumerate(batches):
        if k + 1 < len(batches):
            submit(*batches[k + 1])
        got.append(tile.complete(bid[a:b]))
        gpu_ms.append(tile.last_timing()["gpu_ms"])
    res = np.concatenate([g[0] for g in got]); tag = np.concatenate([g[1] for g in got])
    tsz = np.concatenate([g[2] for g in got])
    assert np.array_equal(tsz, etsz)
    assert np.array_equal(res, eres)
    assert np.array_equal(tag, etag)
    m = tile.metrics()
    assert {k: m[k] for k in o.metrics()} == o.metrics()
    assert m["published"] == int((eres == 0).sum())
    assert len(set(np.unique(res).tolist())) == 5
    # batch latency histograms: one sample per completed batch in each
    from firedancer_amd.verify_tile import hist_edges
    hg, hh = tile.hist("gpu"), tile.hist("host")
    assert int(hg["counts"].sum()) == len(batches) and int(hh["counts"].sum()) == len(batches)
    assert np.array_equal(hg["left_edge_ns"], hist_edges(10_000, 1_000_000_000))
    assert abs(hg["sum_ns"] - sum(round(ms * 1e6) for ms in gpu_ms)) <= len(batches)
    for ms in gpu_ms:                                            # each sample in its bucket
        b = int(np.searchsorted(hg["left_edge_ns"], round(ms * 1e6), side="right")) - 1
        assert hg["counts"][b] > 0
    tile.hist_init(1_000, 50_000_000)
    hg = tile.hist("gpu")
    assert int(hg["counts"].sum()) == 0 and hg["sum_ns"] == 0
    assert np.array_equal(hg["left_edge_ns"], hist_edges(1_000, 50_000_000))
    with pytest.raises(ValueError):
        tile.hist_init(5, 5)
    tile.close()


def test_txn_out_matches_oracle(verifier):
    """fd_txn_t bytes written by the tile's parse for a generated stream."""
    import torch
    from firedancer_amd.txn_workload import make_txn_stream
    s = make_txn_stream(3000, T.oracle_signer, seed=0xabc, bad_frac=0.05)
    tile = _tile(verifier, 1, 1024)
    d = _frags(s.pool, s.off, s.sz)
    d_out = torch.zeros((s.n, 852), dtype=torch.uint8, device="cuda:0")
    res, tag, tsz = tile.after_frags(s.n, *d, txn_out=d_out)
    out = d_out.cpu().numpy()
    etsz, eout = T.oracle_parse_many(s.pool, s.off, s.sz)
    assert np.array_equal(tsz, etsz)
    for j in np.nonzero(etsz)[0]:
        assert np.array_equal(out[j, :etsz[j]], eout[j, :etsz[j]])
    tile.close()
