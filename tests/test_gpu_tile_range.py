"""GPU: the verify tile's mcache range mode (fd_verify_hip_tile_submit_range,
k_range_gather + k_txnm_batch; integration/fd_verify_tile_hip.patch reads an
unpolled quic_verify link this way).

An in-link dcache of fd_txn_m_t frags and an mcache whose lines
(fd_frag_meta_t: seq, sig, chunk, sz, ctl, tsorig, tspub) publish them, as
src/tango/mcache/fd_mcache.h:300-322 lays them out.  A range of seqs goes to
the GPU with a round robin share; the expected outcome is the restated
reference (tests/test_gpu_txn_batch.py's emulate: during_frag's copy and
after_frag's parse, then oracle fd_txn_verify) over exactly the kept seqs in
seq order -- before_frag's filter, fd_verify_tile.c:37-58 -- with each kept
frag's tsorig taken from its line.  Lines the GPU finds reused (a later seq:
the producer lapped the tile) are skipped by the caller's overrun check and
leave no trace; bad ranges are refused."""
import numpy as np
import pytest

import txn_lib as T
from firedancer_amd import verify_tile as V
from test_gpu_txn_batch import PARSED_CHUNKS, _dev, _payloads, emulate, frag_region, stale_out

pytestmark = pytest.mark.gpu

CHUNK_OFF = 37          # link chunk of the dcache's first byte (its wksp offset / 64)


@pytest.fixture(scope="module")
def stream():
    from firedancer_amd.txn_workload import make_txn_stream
    return make_txn_stream(3000, T.oracle_signer, seed=0x7c, dup_frac=0.03, graft_frac=0.01, bad_frac=0.03)


def mcache_lines(depth, seq_base, in_chunk, in_sz, rng):
    """depth lines; seq_base + j publishes frag j (chunk = CHUNK_OFF + in_chunk[j])"""
    m = np.zeros((depth, 4), np.uint64)
    tso = rng.integers(0, 2**32, in_chunk.size, dtype=np.uint64)
    for j in range(in_chunk.size):
        seq = seq_base + j
        w = m[seq & (depth - 1)]
        w[0] = seq
        w[1] = rng.integers(0, 2**63)                                      # sig: not read
        w[2] = (CHUNK_OFF + int(in_chunk[j])) | (int(in_sz[j]) << 32) | (0x3 << 48)
        w[3] = int(tso[j]) | (int(rng.integers(0, 2**32)) << 32)
    return m, tso


def run_range(region, m, depth, seq0, seq_cnt, rr_cnt, rr_idx, out_init, out_chunk, seed, tdepth, skip=None):
    import torch
    n = V.range_frag_cnt(seq0, seq_cnt, rr_cnt, rr_idx)
    tile = V.VerifyTile(None, max_txn=max(n, 1), hashmap_seed=seed, tcache_depth=tdepth, chunk_sigs=1 << 16)
    d_out = _dev(out_init)
    chunk0, wmark = CHUNK_OFF, CHUNK_OFF + region.size // 64 - 40
    got = tile.submit_range(_dev(m.view(np.uint8)), depth, seq0, seq_cnt, rr_cnt, rr_idx, CHUNK_OFF, chunk0, wmark,
                            _dev(region), d_out, _dev(out_chunk, np.int32))
    assert got == n
    res, tsz, psz, tso = tile.complete_range(skip)
    m_ = tile.metrics()
    tile.close()
    tile.verifier.close()
    torch.cuda.synchronize()
    return res, tsz, psz, tso, m_, d_out.cpu().numpy()


def expect(region, in_chunk, in_sz, kinds, out_init, out_chunk, keep_idx, seed, tdepth):
    exp_out, payloads, bids, spans = emulate(region, in_chunk[keep_idx], in_sz[keep_idx], kinds[keep_idx], out_init,
                                             out_chunk)
    pool = np.concatenate(payloads + [np.zeros(1, np.uint8)])
    off = np.cumsum([0] + [p.size for p in payloads[:-1]]).astype(np.uint32)
    sz = np.array([p.size for p in payloads], np.uint16)
    o = T.OracleTile(seed=seed, depth=tdepth)
    eres, _, etsz = o.run(pool, off, sz, bids)
    return exp_out, payloads, spans, eres, etsz, o.metrics()


@pytest.mark.parametrize("rr_cnt,rr_idx,seq0_off", [(1, 0, 0), (3, 1, 5), (4, 3, 2), (6, 0, 7)])
def test_range_equals_kept_seqs(stream, rr_cnt, rr_idx, seq0_off):
    rng = np.random.default_rng(40 + rr_cnt)
    pays = _payloads(stream)[:2400]
    n = len(pays)
    bid = np.zeros(n, np.uint64)
    region, in_chunk, in_sz, kinds = frag_region(pays, bid, np.zeros(n, bool), rng)
    depth, seq_base = 4096, (1 << 40) + 4096 * 3 + 100        # lines wrap the ring; seqs far from 0
    m, tso_all = mcache_lines(depth, seq_base, in_chunk, in_sz, rng)
    seq0, seq_cnt = seq_base + seq0_off, n - seq0_off - 3
    keep_idx = np.array([j for j in range(seq0_off, seq0_off + seq_cnt) if (seq_base + j) % rr_cnt == rr_idx])
    k = keep_idx.size
    out_chunk = (rng.permutation(k) * PARSED_CHUNKS).astype(np.uint32)
    out_init = stale_out(rng, PARSED_CHUNKS * (k + 1), out_chunk)
    res, tsz, psz, tso, mt, out = run_range(region, m, depth, seq0, seq_cnt, rr_cnt, rr_idx, out_init, out_chunk, 17,
                                            1024)
    exp_out, payloads, spans, eres, etsz, em = expect(region, in_chunk, in_sz, kinds, out_init, out_chunk, keep_idx, 17,
                                                      1024)
    assert np.array_equal(res, eres) and np.array_equal(tsz, etsz)
    assert {x: mt[x] for x in em} == em
    assert np.array_equal(tso, tso_all[keep_idx].astype(np.uint32))
    assert np.array_equal(psz, [p.size for p in payloads])
    for sp in spans:
        for a, b in sp:
            assert np.array_equal(out[a:b], exp_out[a:b])
    assert em["dedup_fail_cnt"] + em["verify_fail_cnt"] + em["parse_fail_cnt"] > 0


def test_reused_lines_are_skipped(stream):
    """Lines overwritten by a lapping producer (seq + depth) hold a later seq:
    the GPU flags them without reading their frags, the caller's overrun
    check skips them, and the other frags' outcomes equal the reference run
    over the stream without them."""
    rng = np.random.default_rng(51)
    pays = _payloads(stream)[:1500]
    n = len(pays)
    region, in_chunk, in_sz, kinds = frag_region(pays, np.zeros(n, np.uint64), np.zeros(n, bool), rng)
    depth, seq_base = 2048, 5 * 2048 + 11
    m, _ = mcache_lines(depth, seq_base, in_chunk, in_sz, rng)
    rr_cnt, rr_idx = 2, 1
    keep_idx = np.array([j for j in range(n) if (seq_base + j) % rr_cnt == rr_idx])
    k = keep_idx.size
    lapped = rng.random(k) < 0.15
    for x in np.nonzero(lapped)[0]:
        seq = seq_base + int(keep_idx[x])
        m[seq & (depth - 1), 0] = seq + depth                             # the line of a later frag
        m[seq & (depth - 1), 2] = 0xFFFFFFFF                              # whose chunk is out of range
    out_chunk = (np.arange(k) * PARSED_CHUNKS).astype(np.uint32)
    out_init = stale_out(rng, PARSED_CHUNKS * (k + 1), out_chunk)
    res, tsz, psz, tso, mt, out = run_range(region, m, depth, seq_base, n, rr_cnt, rr_idx, out_init, out_chunk, 23,
                                            512, skip=lapped.astype(np.uint8))
    good = ~lapped
    _, _, _, eres, etsz, em = expect(region, in_chunk, in_sz, kinds, out_init, out_chunk[good], keep_idx[good], 23, 512)
    assert (res[lapped] == V.FRAG_OVERRUN).all()
    assert np.array_equal(res[good], eres) and np.array_equal(tsz[good], etsz)
    assert {x: mt[x] for x in em} == em


def test_bad_ranges_refused(stream):
    import torch
    rng = np.random.default_rng(52)
    pays = _payloads(stream)[:64]
    region, in_chunk, in_sz, _ = frag_region(pays, np.zeros(64, np.uint64), np.zeros(64, bool), rng)
    m, _ = mcache_lines(256, 0, in_chunk, in_sz, rng)
    tile = V.VerifyTile(None, max_txn=64, hashmap_seed=1, tcache_depth=64, chunk_sigs=1 << 16)
    d_m, d_in = _dev(m.view(np.uint8)), _dev(region)
    d_out, oc = _dev(np.zeros(64 * PARSED_CHUNKS * 65, np.uint8)), _dev(np.zeros(512, np.uint32), np.int32)
    wm = CHUNK_OFF + region.size // 64 - 40
    for depth, seq_cnt, rr_cnt, rr_idx, c0, chunk_off in [
            (255, 64, 1, 0, CHUNK_OFF, CHUNK_OFF),       # depth not a power of 2
            (256, 257, 1, 0, CHUNK_OFF, CHUNK_OFF),      # range beyond the ring
            (256, 64, 2, 2, CHUNK_OFF, CHUNK_OFF),       # rr_idx >= rr_cnt
            (256, 64, 1, 0, wm + 1, CHUNK_OFF),          # chunk0 past wmark
            (256, 64, 1, 0, CHUNK_OFF, CHUNK_OFF + 1)]:  # chunk0 before the dcache
        with pytest.raises(RuntimeError):
            tile.submit_range(d_m, depth, 0, seq_cnt, rr_cnt, rr_idx, chunk_off, c0, wm, d_in, d_out, oc)
    with pytest.raises(RuntimeError):                    # a share past max_txn
        tile.submit_range(d_m, 256, 0, 65, 1, 0, CHUNK_OFF, CHUNK_OFF, wm, d_in, d_out, _dev(np.zeros(65, np.int32)))
    assert tile.inflight() == 0
    tile.close()
    tile.verifier.close()
    torch.cuda.synchronize()
