"""GPU: the verify tile fed its own frag format (fd_verify_hip_tile_submit_frags).

The reference's 2048-frag stream fixture (tests/golden/c4_stream_2048.npz:
per-frag results, tags, txn_t_sz, metrics and final tcache arrays of the
reference's after_frag) is re-laid as an in-link dcache of fd_txn_m_t frags
(src/disco/fd_txn_m.h:15-110): 64-B chunks, header with payload_sz and
block_engine.bundle_id, payload after the 80-byte header.  The GPU does
during_frag's copy into the out dcache and after_frag's parse in place; the
results must equal the fixture's, and the out frags must hold the copied
header and payload, txn_t_sz in the header and the fd_txn_t at
fd_txn_m_txn_t (bytes equal to the oracle's parse, itself pinned to the
reference build).

Gossip votes (fd_verify_tile.c:86-98, 112): a share of the non-bundle frags
arrives instead as fd_gossip_update_message_t vote messages; they convert to
fd_txn_m_t (payload_sz = txn_sz, bundle_id 0, source_ipv4, source_tpu =
GOSSIP) and verify exactly as the same payload would; gossiped_votes_cnt
counts them.  A corrupt frag aborts the process, as FD_LOG_ERR ends the
reference tile (child process)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import txn_lib as T
from firedancer_amd import verify_tile as V

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PARSED_CHUNKS = 34     # FD_TPU_PARSED_MTU = 2168 B -> 34 chunks of 64 B


def _dev(a, view=None):
    import torch
    a = np.ascontiguousarray(a)
    if view is not None:
        a = a.view(view)
    return torch.from_numpy(a).to("cuda:0")


def build_in_dcache(pool, off, sz, bundle_id, gossip=None, rng=None):
    """fd_txn_m_t frags (or gossip vote messages where gossip[j]) in 64-B chunks."""
    n = off.size
    gossip = np.zeros(n, bool) if gossip is None else gossip
    rng = rng or np.random.default_rng(1)
    chunks, frags, kinds, sizes, pos = [], [], [], [], 0
    hdr_rand = rng.integers(0, 256, (n, 80), dtype=np.uint8)
    for j in range(n):
        p = pool[off[j]:off[j] + sz[j]]
        if gossip[j]:
            m = rng.integers(0, 256, 80 + 1232, dtype=np.uint8)        # stale union bytes
            m[0] = V.GOSSIP_UPDATE_TAG_VOTE
            m[V.GOSSIP_VOTE_TXN_SZ_OFF:V.GOSSIP_VOTE_TXN_SZ_OFF + 8] = np.frombuffer(np.uint64(sz[j]).tobytes(), np.uint8)
            m[V.GOSSIP_VOTE_TXN_OFF:V.GOSSIP_VOTE_TXN_OFF + sz[j]] = p
            f, kind = m, V.IN_GOSSIP
        else:
            h = hdr_rand[j].copy()
            h[V.TXNM_PAYLOAD_SZ_OFF:V.TXNM_PAYLOAD_SZ_OFF + 2] = np.frombuffer(np.uint16(sz[j]).tobytes(), np.uint8)
            h[V.TXNM_TXN_T_SZ_OFF:V.TXNM_TXN_T_SZ_OFF + 2] = 0xff            # overwritten by the parse
            h[V.TXNM_BUNDLE_ID_OFF:V.TXNM_BUNDLE_ID_OFF + 8] = np.frombuffer(np.uint64(bundle_id[j]).tobytes(), np.uint8)
            f = np.concatenate([h, p])
            kind = V.IN_BUNDLE if bundle_id[j] else V.IN_QUIC
        chunks.append(pos // 64); frags.append(f); kinds.append(kind); sizes.append(f.size)
        pos += (f.size + 63) // 64 * 64 + 64 * int(rng.integers(0, 3))   # gaps between frags
    region = np.zeros(pos + 64, np.uint8)
    for c, f in zip(chunks, frags):
        region[64 * c:64 * c + f.size] = f
    return region, np.array(chunks, np.uint32), np.array(sizes, np.uint16), np.array(kinds, np.uint8), frags


def run_frags(verifier, seed, depth, region, in_chunk, in_sz, kinds, out_chunk, tcache=None):
    import torch
    n = in_chunk.size
    tile = V.VerifyTile(verifier, max_txn=max(n, 1), hashmap_seed=seed, tcache_depth=depth)
    if tcache is not None:
        tile.join_tcache(tcache)
    out_bytes = 64 * (int(out_chunk.max()) + PARSED_CHUNKS) if n else 64
    d_out = torch.full((out_bytes,), 0xa5, dtype=torch.uint8, device="cuda:0")
    tile.submit_frags(n, _dev(region), _dev(in_chunk, np.int32), _dev(in_sz, np.int16), _dev(kinds),
                      d_out, _dev(out_chunk, np.int32))
    res, tag, tsz = tile.complete(None)
    m = tile.metrics()
    tile.close()
    return res, tag, tsz, m, d_out.cpu().numpy()


def check_out_frags(out, out_chunk, frags, kinds, pool, off, sz, tsz, addr=None):
    etsz, eout = T.oracle_parse_many(pool, off, sz)
    assert np.array_equal(tsz, etsz)
    for j, c in enumerate(out_chunk):
        b = 64 * int(c)
        hdr = out[b:b + 80]
        psz = int(hdr[8]) | int(hdr[9]) << 8
        assert psz == sz[j], j
        assert (int(hdr[10]) | int(hdr[11]) << 8) == tsz[j], j
        assert np.array_equal(out[b + 80:b + 80 + psz], pool[off[j]:off[j] + sz[j]]), j
        if kinds[j] == V.IN_GOSSIP:
            assert hdr[V.TXNM_SRC_TPU_OFF] == V.TPU_SOURCE_GOSSIP
            assert hdr[24:32].tobytes() == bytes(8)
            assert hdr[12:16].tobytes() == frags[j][56:60].tobytes()
        else:
            keep = np.ones(80, bool); keep[10:12] = False                 # header copied verbatim but txn_t_sz
            assert np.array_equal(hdr[keep], frags[j][:80][keep]), j
        if tsz[j]:
            t = (b + 80 + psz + 1) // 2 * 2                                 # fd_txn_m_txn_t
            assert np.array_equal(out[t:t + int(tsz[j])], eout[j, :int(tsz[j])]), j


def test_c4_fixture_as_txnm_frags(verifier):
    c4 = dict(np.load(os.path.join(HERE, "golden", "c4_stream_2048.npz")))
    n = c4["off"].size
    region, in_chunk, in_sz, kinds, frags = build_in_dcache(c4["pool"], c4["off"], c4["sz"], c4["bundle_id"])
    out_chunk = (np.random.default_rng(2).permutation(n) * PARSED_CHUNKS).astype(np.uint32)
    tc = V.Tcache(int(c4["depth"]))
    res, tag, tsz, m, out = run_frags(verifier, int(c4["seed"]), int(c4["depth"]), region, in_chunk, in_sz, kinds,
                                      out_chunk, tc)
    assert np.array_equal(res, c4["result"])
    assert np.array_equal(tag, c4["tag"])
    assert np.array_equal(tsz, c4["txn_t_sz"])
    assert [m[k] for k in ("parse_fail_cnt", "verify_fail_cnt", "dedup_fail_cnt", "bundle_peer_fail_cnt")] == \
        c4["metrics"].tolist()
    assert m["gossiped_votes_cnt"] == 0
    assert np.array_equal(tc.ring, c4["ring"]) and np.array_equal(tc.map, c4["map"])
    check_out_frags(out, out_chunk, frags, kinds, c4["pool"], c4["off"], c4["sz"], tsz)


def test_gossip_votes_convert_and_count(verifier):
    c4 = dict(np.load(os.path.join(HERE, "golden", "c4_stream_2048.npz")))
    n = c4["off"].size
    rng = np.random.default_rng(7)
    gossip = (c4["bundle_id"] == 0) & (rng.random(n) < 0.3)
    region, in_chunk, in_sz, kinds, frags = build_in_dcache(c4["pool"], c4["off"], c4["sz"], c4["bundle_id"],
                                                            gossip=gossip, rng=rng)
    out_chunk = (np.arange(n) * PARSED_CHUNKS).astype(np.uint32)
    res, tag, tsz, m, out = run_frags(verifier, int(c4["seed"]), int(c4["depth"]), region, in_chunk, in_sz, kinds,
                                      out_chunk)
    # a gossip vote with bundle_id 0 is processed exactly as the same payload from QUIC
    assert np.array_equal(res, c4["result"]) and np.array_equal(tag, c4["tag"])
    assert m["gossiped_votes_cnt"] == int(gossip.sum()) > 400
    check_out_frags(out, out_chunk, frags, kinds, c4["pool"], c4["off"], c4["sz"], tsz)


def test_generated_stream_vs_oracle_tile(verifier):
    """5000 generated frags (resends, grafted sig0, malformed, bundles) as
    fd_txn_m_t frags against the oracle's after_frag over the same stream."""
    from firedancer_amd.txn_workload import make_txn_stream
    s = make_txn_stream(5000, T.oracle_signer, seed=0x71, dup_frac=0.03, graft_frac=0.01, bad_frac=0.02)
    bid = np.zeros(s.n, np.uint64)
    r = np.random.default_rng(4)
    for start in r.choice(s.n - 8, 60, replace=False):
        bid[start:start + int(r.integers(1, 6))] = int(r.integers(1, 2**40))
    o = T.OracleTile(seed=99, depth=500)
    eres, etag, etsz = o.run(s.pool, s.off, s.sz, bid)
    region, in_chunk, in_sz, kinds, frags = build_in_dcache(s.pool, s.off, s.sz, bid)
    out_chunk = (np.arange(s.n)[::-1] * PARSED_CHUNKS).astype(np.uint32)
    res, tag, tsz, m, out = run_frags(verifier, 99, 500, region, in_chunk, in_sz, kinds, out_chunk)
    assert np.array_equal(tsz, etsz) and np.array_equal(res, eres) and np.array_equal(tag, etag)
    assert {k: m[k] for k in o.metrics()} == o.metrics()


CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/tests")
from firedancer_amd import Verifier, verify_tile as V
v = Verifier(device=0, chunk_sigs=4096)
t = V.VerifyTile(v, max_txn=4, hashmap_seed=1, tcache_depth=16)
f = np.zeros(256, np.uint8); f[8:10] = np.frombuffer(np.uint16(1300).tobytes(), np.uint8)   # payload_sz > FD_TPU_MTU
d = lambda a: torch.from_numpy(a).to("cuda:0")
t.submit_frags(1, d(f), d(np.zeros(1, np.int32)), d(np.array([200], np.int16)), d(np.zeros(1, np.uint8)),
               d(np.zeros(4096, np.uint8)), d(np.zeros(1, np.int32)))
t.complete(None)
print("returned")
"""


def test_corrupt_frag_aborts_like_fd_log_err():
    r = subprocess.run([sys.executable, "-c", CHILD, os.path.dirname(HERE)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == -6, (r.returncode, r.stdout[-500:], r.stderr[-2000:])
    assert "corrupt frag" in r.stderr and "returned" not in r.stdout


def test_zero_copy_ingest_from_mapped_host_memory(verifier):
    """The in-link dcache left in pinned device-mapped host memory
    (fd_ed25519_hip_host_alloc): the ingest kernel reads it in place over PCIe;
    results and out frags equal the HBM-resident run's."""
    import torch
    from firedancer_amd.ed25519 import HostBuffer
    c4 = dict(np.load(os.path.join(HERE, "golden", "c4_stream_2048.npz")))
    n = c4["off"].size
    region, in_chunk, in_sz, kinds, frags = build_in_dcache(c4["pool"], c4["off"], c4["sz"], c4["bundle_id"])
    hb = HostBuffer(region.size)
    hb.array[:] = region
    out_chunk = (np.arange(n) * PARSED_CHUNKS).astype(np.uint32)
    tile = V.VerifyTile(verifier, max_txn=n, hashmap_seed=int(c4["seed"]), tcache_depth=int(c4["depth"]))
    d_out = torch.zeros(64 * (int(out_chunk.max()) + PARSED_CHUNKS), dtype=torch.uint8, device="cuda:0")
    tile.submit_frags(n, hb.ptr, _dev(in_chunk, np.int32), _dev(in_sz, np.int16), _dev(kinds), d_out,
                      _dev(out_chunk, np.int32))
    res, tag, tsz = tile.complete(None)
    tile.close()
    assert np.array_equal(res, c4["result"]) and np.array_equal(tag, c4["tag"])
    check_out_frags(d_out.cpu().numpy(), out_chunk, frags, kinds, c4["pool"], c4["off"], c4["sz"], tsz)
    hb.close()


def test_staged_ingest_from_pinned_host_memory(verifier):
    """The in-link dcache in pinned host memory staged into HBM with
    fd_ed25519_hip_stage_async on the tile's own stream (the DMA copy the C4
    PCIe-inclusive bench leg runs), then submit_frags on the HBM copy; the
    stream orders the copy before the ingest kernel.  Results and out frags
    equal the reference tile's."""
    import torch
    from firedancer_amd.ed25519 import CTX_STREAM, HostBuffer
    c4 = dict(np.load(os.path.join(HERE, "golden", "c4_stream_2048.npz")))
    n = c4["off"].size
    region, in_chunk, in_sz, kinds, frags = build_in_dcache(c4["pool"], c4["off"], c4["sz"], c4["bundle_id"])
    hb = HostBuffer(region.size)
    hb.array[:] = region
    d_in = torch.full((region.size,), 0xA5, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    out_chunk = (np.arange(n) * PARSED_CHUNKS).astype(np.uint32)
    tile = V.VerifyTile(verifier, max_txn=n, hashmap_seed=int(c4["seed"]), tcache_depth=int(c4["depth"]))
    d_out = torch.zeros(64 * (int(out_chunk.max()) + PARSED_CHUNKS), dtype=torch.uint8, device="cuda:0")
    args = (_dev(in_chunk, np.int32), _dev(in_sz, np.int16), _dev(kinds), d_out, _dev(out_chunk, np.int32))
    torch.cuda.synchronize()
    verifier.stage_async(d_in, hb, region.size, stream=CTX_STREAM)
    tile.submit_frags(n, d_in, *args)
    res, tag, tsz = tile.complete(None)
    tile.close()
    assert np.array_equal(d_in.cpu().numpy(), region)
    assert np.array_equal(res, c4["result"]) and np.array_equal(tag, c4["tag"])
    check_out_frags(d_out.cpu().numpy(), out_chunk, frags, kinds, c4["pool"], c4["off"], c4["sz"], tsz)
    hb.close()
