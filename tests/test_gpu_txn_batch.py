"""GPU: k_txnm_batch, the verify tile's one-pass frag kernel (ingest, parse
and record expansion through LDS, firedancer_amd/csrc/fd_txn_hip.hip).

Each test replays the same frags through the reference's byte semantics,
restated here from src/disco/verify/fd_verify_tile.c:64-161:
  during_frag   copy sz bytes of the in frag to the out chunk (or, for a gossip
                vote, write payload_sz / bundle_id / source_ipv4 / source_tpu
                and copy vote.txn);
  after_frag    parse payload_sz bytes of the OUT frag's payload (the stale out
                dcache bytes where the copy did not reach: a header whose
                payload_sz exceeds the frag, a frag shorter than its header),
                write txn_t_sz into the out header and the fd_txn_t at
                fd_txn_m_txn_t; then fd_txn_verify (oracle tile, pinned to the
                reference build by tests/test_ref_fixture.py).
and checks per-frag results, tags, metrics and the out dcache's bytes, and
that the split three-kernel form (FD_VERIFY_HIP_INGEST=split) and both group
sizes (FD_VERIFY_HIP_FB=8/16) write the same out dcache byte for byte, as
does out staging (fd_verify_hip_tile_set_staging: the batch on HBM staging
frags, then only the bytes the reference writes copied to the out dcache)."""
import os

import numpy as np
import pytest

import txn_lib as T
from firedancer_amd import verify_tile as V

pytestmark = pytest.mark.gpu

PARSED_CHUNKS = 34     # FD_TPU_PARSED_MTU = 2168 B in 64-B chunks


def _dev(a, view=None):
    import torch
    a = np.ascontiguousarray(a)
    if view is not None:
        a = a.view(view)
    return torch.from_numpy(a).to("cuda:0")


def _u16(b):
    return int(b[0]) | int(b[1]) << 8


def stale_out(rng, n_chunks, out_chunk):
    """a random out dcache whose stale headers hold payload_sz <= FD_TPU_MTU
    (a frag shorter than 10 bytes takes payload_sz from them)"""
    out = rng.integers(0, 256, 64 * n_chunks, dtype=np.uint8)
    for c in out_chunk:
        out[64 * int(c) + 8:64 * int(c) + 10] = np.frombuffer(np.uint16(rng.integers(0, 1233)).tobytes(), np.uint8)
    return out


def emulate(region_in, in_chunk, in_sz, kinds, out_init, out_chunk, in_place=False):
    """during_frag + after_frag's parse on numpy buffers; returns the out
    dcache, the payload each frag's parse read, bundle ids and the ranges of
    out bytes the reference defines (header, payload, fd_txn_t)."""
    out = out_init.copy()
    src = out if in_place else region_in
    payloads, bids, spans = [], [], []
    for j in range(in_chunk.size):
        i0, o0, sz = 64 * int(in_chunk[j]), 64 * int(out_chunk[j]), int(in_sz[j])
        if kinds[j] == V.IN_GOSSIP:
            psz = int(np.frombuffer(src[i0 + 72:i0 + 80].tobytes(), np.uint64)[0])
            out[o0 + 8:o0 + 10] = np.frombuffer(np.uint16(psz).tobytes(), np.uint8)
            out[o0 + 24:o0 + 32] = 0
            out[o0 + 12:o0 + 16] = src[i0 + 56:i0 + 60]
            out[o0 + 16] = V.TPU_SOURCE_GOSSIP
            out[o0 + 80:o0 + 80 + psz] = src[i0 + 80:i0 + 80 + psz]
            bid = 0
            hdr_keep = [(8, 10), (12, 17), (24, 32)]
        else:
            if not in_place:
                out[o0:o0 + sz] = src[i0:i0 + sz]
            psz = _u16(out[o0 + 8:o0 + 10])
            bid = int(np.frombuffer(out[o0 + 24:o0 + 32].tobytes(), np.uint64)[0])
            hdr_keep = [(0, 10), (12, 80)]
        assert psz <= 1232, (j, psz)            # else a corrupt frag: the test's construction is wrong
        payload = out[o0 + 80:o0 + 80 + psz].copy()
        tsz, txn_t = T.oracle_parse(payload)
        out[o0 + 10:o0 + 12] = np.frombuffer(np.uint16(tsz).tobytes(), np.uint8)
        sp = [(o0 + a, o0 + b) for a, b in hdr_keep] + [(o0 + 10, o0 + 12), (o0 + 80, o0 + 80 + psz)]
        if tsz:
            t = o0 + (80 + psz + 1) // 2 * 2
            out[t:t + tsz] = np.frombuffer(txn_t, np.uint8)
            sp.append((t, t + tsz))
        payloads.append(payload)
        bids.append(bid)
        spans.append(sp)
    return out, payloads, np.array(bids, np.uint64), spans


def run_tile(region_in, in_chunk, in_sz, kinds, out_init, out_chunk, seed, depth, in_place=False, env=None,
             staging=False):
    import torch
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        n = in_chunk.size
        tile = V.VerifyTile(None, max_txn=max(n, 1), hashmap_seed=seed, tcache_depth=depth, chunk_sigs=1 << 16)
        if staging:
            tile.set_staging(True)
        d_out = _dev(out_init)
        d_in = d_out if in_place else _dev(region_in)
        tile.submit_frags(n, d_in, _dev(in_chunk, np.int32), _dev(in_sz, np.int16), _dev(kinds), d_out,
                          _dev(out_chunk, np.int32))
        res, tag, tsz = tile.complete(None)
        m = tile.metrics()
        tile.close()
        tile.verifier.close()
        torch.cuda.synchronize()
        return res, tag, tsz, m, d_out.cpu().numpy()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def check(res, tag, tsz, m, out, exp_out, payloads, bids, spans, seed, depth, out_init):
    pool = np.concatenate(payloads + [np.zeros(1, np.uint8)])
    off = np.cumsum([0] + [p.size for p in payloads[:-1]]).astype(np.uint32)
    sz = np.array([p.size for p in payloads], np.uint16)
    o = T.OracleTile(seed=seed, depth=depth)
    eres, etag, etsz = o.run(pool, off, sz, bids)
    assert np.array_equal(tsz, etsz)
    assert np.array_equal(res, eres)
    assert np.array_equal(tag, etag)
    assert {k: m[k] for k in o.metrics()} == o.metrics()
    for j, sp in enumerate(spans):
        for a, b in sp:
            assert np.array_equal(out[a:b], exp_out[a:b]), (j, a, b)
    # nothing outside the frags' out chunks is written
    touched = np.zeros(out.size, bool)
    for sp in spans:
        lo = min(a for a, _ in sp) // 64 * 64
        touched[lo:lo + 64 * PARSED_CHUNKS] = True
    assert np.array_equal(out[~touched], out_init[~touched])


def frag_region(payloads, bid, gossip, rng, hdr_psz=None, frag_sz=None):
    """in-link dcache of fd_txn_m_t frags / gossip votes, 64-B chunks with gaps;
    hdr_psz / frag_sz override the header's payload_sz and the mcache size."""
    n = len(payloads)
    chunks, kinds, sizes, frags, pos = [], [], [], [], 0
    for j in range(n):
        p = payloads[j]
        if gossip[j]:
            f = rng.integers(0, 256, 80 + 1232, dtype=np.uint8)
            f[0] = V.GOSSIP_UPDATE_TAG_VOTE
            f[72:80] = np.frombuffer(np.uint64(p.size).tobytes(), np.uint8)
            f[80:80 + p.size] = p
            kind, fs = V.IN_GOSSIP, int(rng.integers(80 + p.size, 2049))
        else:
            h = rng.integers(0, 256, 80, dtype=np.uint8)
            ps = p.size if hdr_psz is None or hdr_psz[j] is None else hdr_psz[j]
            h[8:10] = np.frombuffer(np.uint16(ps).tobytes(), np.uint8)
            h[24:32] = np.frombuffer(np.uint64(bid[j]).tobytes(), np.uint8)
            f = np.concatenate([h, p])
            kind = V.IN_BUNDLE if bid[j] else V.IN_QUIC
            fs = f.size if frag_sz is None or frag_sz[j] is None else frag_sz[j]
        chunks.append(pos // 64); kinds.append(kind); sizes.append(fs); frags.append(f)
        pos += (max(f.size, fs) + 63) // 64 * 64 + 64 * int(rng.integers(0, 3))
    region = rng.integers(0, 256, pos + 4096, dtype=np.uint8)           # bytes past a frag are not zero
    for c, f in zip(chunks, frags):
        region[64 * c:64 * c + f.size] = f
    return region, np.array(chunks, np.uint32), np.array(sizes, np.uint16), np.array(kinds, np.uint8)


@pytest.fixture(scope="module")
def stream():
    from firedancer_amd.txn_workload import make_txn_stream
    return make_txn_stream(6000, T.oracle_signer, seed=0x7b, dup_frac=0.03, graft_frac=0.01, bad_frac=0.03)


def _payloads(s):
    return [s.pool[int(s.off[j]):int(s.off[j]) + int(s.sz[j])].copy() for j in range(s.n)]


def test_generated_stream_all_forms(stream):
    """6000 generated frags (resends, grafts, malformed), bundles and 15%
    gossip votes: the fused kernel at both group sizes and the split form
    against the restated reference; the three out dcaches are byte-equal."""
    rng = np.random.default_rng(11)
    s = stream
    pays = _payloads(s)
    bid = np.zeros(s.n, np.uint64)
    for start in rng.choice(s.n - 8, 80, replace=False):
        bid[start:start + int(rng.integers(1, 6))] = int(rng.integers(1, 2**40))
    gossip = (bid == 0) & (rng.random(s.n) < 0.15)
    region, in_chunk, in_sz, kinds = frag_region(pays, bid, gossip, rng)
    out_chunk = (rng.permutation(s.n) * PARSED_CHUNKS).astype(np.uint32)
    out_init = stale_out(rng, PARSED_CHUNKS * (s.n + 1), out_chunk)
    exp_out, payloads, bids, spans = emulate(region, in_chunk, in_sz, kinds, out_init, out_chunk)
    outs = []
    for env in ({}, {"FD_VERIFY_HIP_FB": "8"}, {"FD_VERIFY_HIP_INGEST": "split"}):
        r = run_tile(region, in_chunk, in_sz, kinds, out_init, out_chunk, 77, 700, env=env)
        check(*r, exp_out, payloads, bids, spans, 77, 700, out_init)
        outs.append(r[4])
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])


@pytest.mark.parametrize("n", [1, 7, 15, 16, 17, 33, 64, 65])
def test_ragged_batches(stream, n):
    rng = np.random.default_rng(n)
    pays = _payloads(stream)[:n]
    bid = np.zeros(n, np.uint64)
    gossip = rng.random(n) < 0.2
    region, in_chunk, in_sz, kinds = frag_region(pays, bid, gossip, rng)
    out_chunk = (np.arange(n) * PARSED_CHUNKS).astype(np.uint32)
    out_init = stale_out(rng, PARSED_CHUNKS * (n + 1), out_chunk)
    exp_out, payloads, bids, spans = emulate(region, in_chunk, in_sz, kinds, out_init, out_chunk)
    r = run_tile(region, in_chunk, in_sz, kinds, out_init, out_chunk, 5, 64)
    check(*r, exp_out, payloads, bids, spans, 5, 64, out_init)


@pytest.mark.parametrize("staging", [False, True])
def test_lying_headers_and_short_frags(stream, staging):
    """Headers whose payload_sz is below or above the frag's bytes (the parse
    then reads stale out-dcache bytes, as after_frag does), frags shorter
    than their 80-B header, and a header-only frag; in place and with out
    staging (whose verify then hashes those stale bytes from the staging
    frag)."""
    rng = np.random.default_rng(3)
    pays = _payloads(stream)[:400]
    n = len(pays)
    hdr_psz, frag_sz = [None] * n, [None] * n
    for j in range(n):
        k = j % 8
        p = pays[j].size
        if k == 1:
            hdr_psz[j] = max(0, p - int(rng.integers(1, 40)))                 # payload_sz < copied payload
        elif k == 2:
            hdr_psz[j] = min(1232, p + int(rng.integers(1, 200)))             # payload_sz > copied payload
        elif k == 3:
            frag_sz[j] = int(rng.integers(1, 80))                             # frag shorter than its header
        elif k == 4:
            frag_sz[j] = 80                                                   # header only
        elif k == 5:
            frag_sz[j] = 80 + p - int(rng.integers(1, min(p, 64) + 1))       # truncated copy
    bid = np.zeros(n, np.uint64)
    gossip = np.zeros(n, bool)
    region, in_chunk, in_sz, kinds = frag_region(pays, bid, gossip, rng, hdr_psz, frag_sz)
    out_chunk = (rng.permutation(n) * PARSED_CHUNKS).astype(np.uint32)
    out_init = stale_out(rng, PARSED_CHUNKS * (n + 1), out_chunk)
    exp_out, payloads, bids, spans = emulate(region, in_chunk, in_sz, kinds, out_init, out_chunk)
    # the stale-byte cases are exercised: some frags parse bytes the copy never wrote
    assert sum(1 for j in range(n) if payloads[j].size + 80 > int(in_sz[j])) >= 100
    r = run_tile(region, in_chunk, in_sz, kinds, out_init, out_chunk, 9, 256, staging=staging)
    check(*r, exp_out, payloads, bids, spans, 9, 256, out_init)
    assert (r[0] == V.FRAG_PUBLISH).sum() > 50 and (r[0] == V.FRAG_PARSE_FAIL).sum() > 50


def test_in_place_frags(stream):
    """in chunk == out chunk (the patched reference tile's own during_frag has
    copied the frag): nothing is copied, the parse reads the frag in place,
    including bytes past the staged pieces for a lying payload_sz."""
    rng = np.random.default_rng(4)
    pays = _payloads(stream)[:300]
    n = len(pays)
    hdr_psz = [min(1232, p.size + int(rng.integers(1, 100))) if j % 5 == 0 else None for j, p in enumerate(pays)]
    bid = np.zeros(n, np.uint64)
    region, in_chunk, in_sz, kinds = frag_region(pays, bid, np.zeros(n, bool), rng, hdr_psz)
    # lay the frags out at PARSED_CHUNKS strides in one buffer that is both the in and the out dcache
    chunk = (np.arange(n) * PARSED_CHUNKS).astype(np.uint32)
    buf = stale_out(rng, PARSED_CHUNKS * (n + 1), chunk)
    for j in range(n):
        a = 64 * int(in_chunk[j])
        buf[64 * int(chunk[j]):64 * int(chunk[j]) + int(in_sz[j])] = region[a:a + int(in_sz[j])]
    exp_out, payloads, bids, spans = emulate(None, chunk, in_sz, kinds, buf, chunk, in_place=True)
    r = run_tile(None, chunk, in_sz, kinds, buf, chunk, 13, 128, in_place=True)
    check(*r, exp_out, payloads, bids, spans, 13, 128, buf)


def test_host_copied_and_gpu_copied_frags(stream):
    """A batch mixing the two sources the patched tile uses with
    FD_VERIFY_HIP_GPU_COPY: frags the host tile's during_frag already copied
    into their out chunks (kind | FD_VERIFY_HIP_IN_HOSTCOPY, in chunk
    garbage) and frags the GPU copies from the in dcache, gossip votes and
    lying headers among them, against the restated reference, every group
    size and the split form byte-equal."""
    rng = np.random.default_rng(12)
    s = stream
    pays = _payloads(s)[:2000]
    n = len(pays)
    bid = np.zeros(n, np.uint64)
    gossip = rng.random(n) < 0.1
    hdr_psz = [min(1232, p.size + int(rng.integers(1, 100))) if j % 9 == 0 and not gossip[j] else None
               for j, p in enumerate(pays)]
    region, in_chunk, in_sz, kinds = frag_region(pays, bid, gossip, rng, hdr_psz)
    out_chunk = (rng.permutation(n) * PARSED_CHUNKS).astype(np.uint32)
    out_init = stale_out(rng, PARSED_CHUNKS * (n + 1), out_chunk)
    exp_out, payloads, bids, spans = emulate(region, in_chunk, in_sz, kinds, out_init, out_chunk)
    host = (rng.random(n) < 0.5) & (kinds != V.IN_GOSSIP)
    pre = out_init.copy()                      # the host tile's during_frag for those frags
    for j in np.nonzero(host)[0]:
        a, o, z = 64 * int(in_chunk[j]), 64 * int(out_chunk[j]), int(in_sz[j])
        pre[o:o + z] = region[a:a + z]
    k2 = kinds.copy()
    k2[host] |= V.IN_HOSTCOPY
    ic2 = in_chunk.copy()
    ic2[host] = 0xFFFFFFF0                     # never read
    outs = []
    for env in ({}, {"FD_VERIFY_HIP_FB": "8"}, {"FD_VERIFY_HIP_INGEST": "split"}):
        r = run_tile(region, ic2, in_sz, k2, pre, out_chunk, 91, 4096, env=env)
        check(*r, exp_out, payloads, bids, spans, 91, 4096, pre)
        outs.append(r[4])
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
    assert host.sum() > 0.3 * n and r[3]["gossiped_votes_cnt"] == int(gossip.sum())


def test_overrun_skip_is_invisible(stream):
    """complete_skip: frags the caller found overrun (the GPU-copy tile's
    post-read mcache check) get FRAG_OVERRUN and leave no trace in the
    ordered pass -- the others' results, tags, metrics and tcache equal the
    reference run over the stream without them (the stream's resends make a
    leaked tcache insert visible as an extra dedup)."""
    import torch
    rng = np.random.default_rng(13)
    pays = _payloads(stream)[:1500]
    n = len(pays)
    bid = np.zeros(n, np.uint64)
    for start in rng.choice(n - 8, 20, replace=False):
        bid[start:start + int(rng.integers(1, 6))] = int(rng.integers(1, 2**40))
    region, in_chunk, in_sz, kinds = frag_region(pays, bid, np.zeros(n, bool), rng)
    out_chunk = (np.arange(n) * PARSED_CHUNKS).astype(np.uint32)
    out_init = stale_out(rng, PARSED_CHUNKS * (n + 1), out_chunk)
    skip = rng.random(n) < 0.2
    keep = ~skip
    _, payloads, bids, _ = emulate(region, in_chunk[keep], in_sz[keep], kinds[keep], out_init, out_chunk[keep])
    tile = V.VerifyTile(None, max_txn=n, hashmap_seed=5, tcache_depth=512, chunk_sigs=1 << 16)
    tile.submit_frags(n, _dev(region), _dev(in_chunk, np.int32), _dev(in_sz, np.int16), _dev(kinds), _dev(out_init),
                      _dev(out_chunk, np.int32))
    res, tag, tsz = tile.complete_skip(skip.astype(np.uint8))
    psz = tile.last_payload_sz
    m = tile.metrics()
    tile.close()
    tile.verifier.close()
    torch.cuda.synchronize()
    pool = np.concatenate(payloads + [np.zeros(1, np.uint8)])
    off = np.cumsum([0] + [p.size for p in payloads[:-1]]).astype(np.uint32)
    sz = np.array([p.size for p in payloads], np.uint16)
    o = T.OracleTile(seed=5, depth=512)
    eres, etag, etsz = o.run(pool, off, sz, bids)
    assert (res[skip] == V.FRAG_OVERRUN).all() and (tag[skip] == 0).all()
    assert np.array_equal(res[keep], eres) and np.array_equal(tag[keep], etag) and np.array_equal(tsz[keep], etsz)
    assert {k: m[k] for k in o.metrics()} == o.metrics()
    assert o.metrics()["dedup_fail_cnt"] > 0
    assert np.array_equal(psz[keep], [p.size for p in payloads])    # the out headers' payload_sz


def test_large_batch_records_and_order(stream):
    """A 2^16-frag batch (the generated stream tiled, each frag re-keyed so no
    resend is a dedup of another copy's): every signature gets a record
    (the survivor count equals the stream's), verdicts equal the split
    form's."""
    import torch  # noqa: F401
    rng = np.random.default_rng(6)
    s = stream
    pays = _payloads(s)
    reps = (1 << 16) // s.n + 1
    pays = (pays * reps)[:1 << 16]
    n = len(pays)
    bid = np.zeros(n, np.uint64)
    region, in_chunk, in_sz, kinds = frag_region(pays, bid, np.zeros(n, bool), rng)
    out_chunk = (np.arange(n) * PARSED_CHUNKS).astype(np.uint32)
    out_init = np.zeros(64 * PARSED_CHUNKS * (n + 1), np.uint8)
    a = run_tile(region, in_chunk, in_sz, kinds, out_init, out_chunk, 21, 1 << 17)
    b = run_tile(region, in_chunk, in_sz, kinds, out_init, out_chunk, 21, 1 << 17,
                 env={"FD_VERIFY_HIP_INGEST": "split"})
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x, y)
    assert a[3] == b[3]
    assert np.array_equal(a[4], b[4])
    assert a[3]["sigs"] == b[3]["sigs"] > n


def test_groups_over_the_lds_budget(stream):
    """Groups whose pieces overflow k_txnm_batch's LDS budget (16 frags of
    700-1232 B) take the global path; interleaved with normal groups, and
    with gossip votes among them."""
    rng = np.random.default_rng(8)
    pays = _payloads(stream)
    big = [p for p in pays if p.size >= 700]
    small = [p for p in pays if p.size < 700]
    assert len(big) >= 160
    order = big[:96] + small[:64] + big[96:160] + small[64:100]
    n = len(order)
    bid = np.zeros(n, np.uint64)
    gossip = rng.random(n) < 0.1
    region, in_chunk, in_sz, kinds = frag_region(order, bid, gossip, rng)
    out_chunk = (rng.permutation(n) * PARSED_CHUNKS).astype(np.uint32)
    out_init = stale_out(rng, PARSED_CHUNKS * (n + 1), out_chunk)
    exp_out, payloads, bids, spans = emulate(region, in_chunk, in_sz, kinds, out_init, out_chunk)
    r = run_tile(region, in_chunk, in_sz, kinds, out_init, out_chunk, 31, 512)
    check(*r, exp_out, payloads, bids, spans, 31, 512, out_init)
    s = run_tile(region, in_chunk, in_sz, kinds, out_init, out_chunk, 31, 512, env={"FD_VERIFY_HIP_INGEST": "split"})
    assert np.array_equal(r[4], s[4])


def test_out_staging_writes_the_same_bytes(stream):
    """Out staging against the in-place form on every frag shape the other
    tests use -- gossip votes, bundles, host-copied frags, headers whose
    payload_sz runs past the frag, frags shorter than their header, groups
    over the LDS budget -- in one batch: results, tags, metrics and the out
    dcache are equal byte for byte (the flush writes exactly the reference's
    bytes; a staging frag's payload past the copy comes from the out dcache's
    own bytes), and both equal the restated reference.  One exception, never
    published: a failed parse leaves the fields it wrote before failing in
    the in-place out dcache (as fd_txn_parse.c:133-180 does in the
    reference's), and staging does not flush a failed parse's fd_txn_t."""
    rng = np.random.default_rng(14)
    pays = _payloads(stream)[:3000]
    big = [p for p in pays if p.size >= 700][:64]
    pays = pays[:1500] + big + pays[1500:2900]
    n = len(pays)
    bid = np.zeros(n, np.uint64)
    for start in rng.choice(n - 8, 40, replace=False):
        bid[start:start + int(rng.integers(1, 6))] = int(rng.integers(1, 2**40))
    gossip = (bid == 0) & (rng.random(n) < 0.1)
    hdr_psz = [min(1232, p.size + int(rng.integers(1, 100))) if j % 11 == 0 and not gossip[j] else None
               for j, p in enumerate(pays)]
    frag_sz = [int(rng.integers(1, 80)) if j % 97 == 5 and not gossip[j] else None for j in range(n)]
    region, in_chunk, in_sz, kinds = frag_region(pays, bid, gossip, rng, hdr_psz, frag_sz)
    out_chunk = (rng.permutation(n) * PARSED_CHUNKS).astype(np.uint32)
    out_init = stale_out(rng, PARSED_CHUNKS * (n + 1), out_chunk)
    exp_out, payloads, bids, spans = emulate(region, in_chunk, in_sz, kinds, out_init, out_chunk)
    host = (rng.random(n) < 0.3) & (kinds != V.IN_GOSSIP)
    pre = out_init.copy()
    for j in np.nonzero(host)[0]:
        a, o, z = 64 * int(in_chunk[j]), 64 * int(out_chunk[j]), int(in_sz[j])
        pre[o:o + z] = region[a:a + z]
    k2 = kinds.copy()
    k2[host] |= V.IN_HOSTCOPY
    ic2 = in_chunk.copy()
    ic2[host] = 0xFFFFFFF0
    a = run_tile(region, ic2, in_sz, k2, pre, out_chunk, 93, 4096)
    b = run_tile(region, ic2, in_sz, k2, pre, out_chunk, 93, 4096, staging=True)
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x, y)
    assert a[3] == b[3]
    keep = np.ones(a[4].size, bool)
    for j in np.nonzero(a[2] == 0)[0]:                  # a failed parse's partial fd_txn_t
        t = 64 * int(out_chunk[j]) + (80 + payloads[j].size + 1) // 2 * 2
        keep[t:t + 852] = False
    assert np.array_equal(a[4][keep], b[4][keep])
    assert (~keep).sum() > 0 and keep.sum() > 0.9 * keep.size
    check(*b, exp_out, payloads, bids, spans, 93, 4096, pre)
    assert a[3]["parse_fail_cnt"] > 0 and a[3]["gossiped_votes_cnt"] == int(gossip.sum())


def test_out_staging_refused_under_split(stream):
    tile = V.VerifyTile(None, max_txn=16, hashmap_seed=1, tcache_depth=64, chunk_sigs=1 << 16)
    tile.set_staging(True)
    tile.set_staging(False)
    tile.close()
    tile.verifier.close()
    old = os.environ.get("FD_VERIFY_HIP_INGEST")
    os.environ["FD_VERIFY_HIP_INGEST"] = "split"
    try:
        tile = V.VerifyTile(None, max_txn=16, hashmap_seed=1, tcache_depth=64, chunk_sigs=1 << 16)
        with pytest.raises(ValueError):
            tile.set_staging(True)
        tile.close()
        tile.verifier.close()
    finally:
        if old is None:
            os.environ.pop("FD_VERIFY_HIP_INGEST", None)
        else:
            os.environ["FD_VERIFY_HIP_INGEST"] = old
