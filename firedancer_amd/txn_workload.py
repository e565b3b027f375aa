"""Synthetic Solana transaction stream for config C4 (verify tile), repo-owned.

SURVEY.md 8(d) C4: legacy/v0 transactions in the shape of the reference's
benchg templates (src/app/shared_dev/commands/bench/fd_benchg.c:71-166:
fee payer(s), a destination and a program account, a recent blockhash, one
instruction), extended to 1-12 signers:

  signers        80% 1, 10% 2, 5% 3-6, 5% 7-12
  version        90% legacy, 10% v0 with one address-table lookup
  body           75% transfer-like (9 data bytes), 25% padded to a random
                 size up to FD_TXN_MTU (1232 B, like large_noop_t)
  validity       the C2 mutation model per signature (workload.c2_mutate)
  duplicates     1% exact resends of an earlier txn (same sig0 -> dedup)
                 0.1% another txn's sig0 grafted onto a different body
  malformed      0.5% (truncated, sig count mismatch, zero signatures)

Every signer signs the txn message payload[1+64n:] (fd_txn.h: message_off).
Signing goes through a caller-supplied signer: the oracle for CPU tests, the
engine's GPU signer (fd_ed25519_hip_sign_dev) for the bench.
"""
from dataclasses import dataclass

import numpy as np

from .workload import c2_mutate

MTU = 1232


@dataclass
class TxnStream:
    pool: np.ndarray       # uint8 payload bytes
    off: np.ndarray        # uint32 per frag, arrival order
    sz: np.ndarray         # uint16 per frag
    nsig: np.ndarray       # uint8 declared signature count per frag (before malformation)
    n_records: int         # signatures signed

    @property
    def n(self):
        return int(self.off.shape[0])


def _cu16(v):
    return [v] if v < 0x80 else [(v & 0x7f) | 0x80, v >> 7]


def _size(n, e, v0, d):
    return 1 + 64 * n + (4 if v0 else 3) + 1 + 32 * (n + e) + 32 + 1 + 1 + 1 + e + len(_cu16(d)) + d + (37 if v0 else 0)


def _shape(rng, n, large, v0_frac=0.10):
    """(extra accounts e, v0, data size d) for a txn with n signers that fits the MTU."""
    e, v0, d = 2, bool(rng.random() < v0_frac), 9
    while _size(n, e, v0, d) > MTU:
        if v0:
            v0 = False
        elif e == 2:
            e = 1
        else:
            d = max(0, d - (_size(n, e, v0, d) - MTU))
    if large:
        lo = _size(n, e, v0, d)
        target = int(rng.integers(lo, MTU + 1))
        d2 = d + (target - lo)
        while _size(n, e, v0, d2) > target:
            d2 -= 1
        d = max(d, d2)
    return e, v0, d


def _nsig(rng, k):
    u = rng.random(k)
    return np.where(u < 0.80, 1, np.where(u < 0.90, 2, np.where(u < 0.95, rng.integers(3, 7, k),
                                                                rng.integers(7, 13, k)))).astype(np.int64)


def make_txn_stream(n_txn, signer, seed=0x5eed0004, mix="c2", dup_frac=0.01, graft_frac=0.001, bad_frac=0.005,
                    v0_frac=0.10):
    """Build n_txn frags; signer(prvs[m,32], pool, msg_off, msg_sz) -> (pubs, sigs).
    mix "c2" applies the C2 mutation model, anything else keeps every
    signature valid; v0_frac is the share of v0 txns (each with one
    address-table lookup)."""
    rng = np.random.default_rng(seed)
    nsig = _nsig(rng, n_txn)
    large = rng.random(n_txn) < 0.25
    shapes = [_shape(rng, int(nsig[t]), bool(large[t]), v0_frac) for t in range(n_txn)]
    keys = np.array([(nsig[t], s[0], int(s[1]), s[2]) for t, s in enumerate(shapes)], np.int64)
    size = np.array([_size(int(k[0]), int(k[1]), bool(k[2]), int(k[3])) for k in keys], np.int64)
    off = np.zeros(n_txn, np.int64)
    pool = np.zeros(int(size.sum()) + 64, np.uint8)
    msg_at = np.zeros(n_txn, np.int64)
    acct_at = np.zeros(n_txn, np.int64)

    # payloads of one shape are built as one (count, size) matrix and laid out
    # contiguously; arrival order is a permutation applied afterwards
    uk, inv = np.unique(keys, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    gbase = 0
    for g, (n, e, v0, d) in enumerate(uk):
        n, e, v0, d = int(n), int(e), bool(v0), int(d)
        rows = np.nonzero(inv == g)[0]
        c, S = rows.size, _size(n, e, v0, d)
        M = np.zeros((c, S), np.uint8)
        M[:, 0] = n
        o = 1 + 64 * n
        mo = o
        if v0:
            M[:, o] = 0x80; o += 1
        M[:, o:o + 3] = (n, 0, 1); o += 3                   # sig cnt, ro_signed, ro_unsigned (the program)
        M[:, o] = n + e; o += 1                              # acct_addr_cnt (compact-u16, < 128)
        ao = o
        M[:, o + 32 * n:o + 32 * (n + e) + 32] = rng.integers(0, 256, (c, 32 * e + 32), dtype=np.uint8)
        o += 32 * (n + e) + 32                               # accounts + recent blockhash
        M[:, o] = 1; o += 1                                  # instr_cnt
        M[:, o] = n + e - 1; o += 1                          # program id = last account
        ia = [0, n] if e == 2 else [0]
        M[:, o] = len(ia); o += 1
        M[:, o:o + len(ia)] = ia; o += len(ia)
        cu = _cu16(d)
        M[:, o:o + len(cu)] = cu; o += len(cu)
        M[:, o:o + d] = rng.integers(0, 256, (c, d), dtype=np.uint8); o += d
        if v0:                                               # one lookup: 1 writable + 1 readonly index
            M[:, o] = 1; o += 1
            M[:, o:o + 32] = rng.integers(0, 256, (c, 32), dtype=np.uint8); o += 32
            M[:, o] = 1; M[:, o + 1] = rng.integers(0, 256, c); o += 2
            M[:, o] = 1; M[:, o + 1] = rng.integers(0, 256, c); o += 2
        assert o == S, (o, S)
        off[rows] = gbase + S * np.arange(c)
        pool[gbase:gbase + c * S] = M.reshape(-1)
        gbase += c * S
        msg_at[rows] = off[rows] + mo
        acct_at[rows] = off[rows] + ao

    # signature records: txn t, signer k
    rec_t = np.repeat(np.arange(n_txn), nsig)
    rec_k = np.arange(rec_t.size) - np.repeat(np.cumsum(nsig) - nsig, nsig)
    m = rec_t.size
    sig_at = off[rec_t] + 1 + 64 * rec_k
    pub_at = acct_at[rec_t] + 32 * rec_k
    prvs = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    zero = np.zeros(m, np.uint32)
    pubs, _ = signer(prvs, np.zeros(16, np.uint8), zero, zero)
    pool[pub_at[:, None] + np.arange(32)] = pubs
    msz = (off[rec_t] + size[rec_t] - msg_at[rec_t]).astype(np.uint32)
    _, sigs = signer(prvs, pool, msg_at[rec_t].astype(np.uint32), msz)
    sigs = np.array(sigs, np.uint8)
    pubs = np.array(pubs, np.uint8)
    if mix == "c2":
        c2_mutate(sigs, pubs, rng)
    pool[sig_at[:, None] + np.arange(64)] = sigs
    pool[pub_at[:, None] + np.arange(32)] = pubs

    # arrival order, resends, grafted sig0, malformed frags
    order = rng.permutation(n_txn)
    f_off, f_sz, f_n = off[order].copy(), size[order].copy(), nsig[order].copy()
    for j in np.nonzero(rng.random(n_txn) < dup_frac)[0]:
        if j == 0:
            continue
        src = j - 1 - int(rng.integers(0, min(j, 4096)))
        f_off[j], f_sz[j], f_n[j] = f_off[src], f_sz[src], f_n[src]
    def append(pool, bodies):
        if not bodies:
            return pool, []
        offs = pool.size + np.concatenate([[0], np.cumsum([b.size for b in bodies])[:-1]])
        return np.concatenate([pool] + bodies), list(offs)

    bodies, who = [], []
    for j in np.nonzero(rng.random(n_txn) < graft_frac)[0]:
        if j == 0:
            continue
        src = j - 1 - int(rng.integers(0, min(j, 4096)))
        body = pool[f_off[j]:f_off[j] + f_sz[j]].copy()
        body[1:65] = pool[f_off[src] + 1:f_off[src] + 65]
        bodies.append(body); who.append(j)
    pool, offs = append(pool, bodies)
    f_off[who] = offs
    bodies, who = [], []
    for j in np.nonzero(rng.random(n_txn) < bad_frac)[0]:
        body = pool[f_off[j]:f_off[j] + f_sz[j]].copy()
        kind = int(rng.integers(0, 3))
        if kind == 0:
            body = body[:-1 - int(rng.integers(0, 8))]       # truncated
        elif kind == 1:
            body[1 + 64 * int(body[0])] ^= 0x01              # header sig count != sig count
        else:
            body[0] = 0                                      # no fee payer
        bodies.append(body); who.append(j)
    pool, offs = append(pool, bodies)
    f_off[who] = offs
    f_sz[who] = [b.size for b in bodies]
    pool = np.concatenate([pool, np.zeros(64, np.uint8)])
    return TxnStream(pool=pool, off=f_off.astype(np.uint32), sz=f_sz.astype(np.uint16), nsig=f_n.astype(np.uint8),
                     n_records=int(m))


def gpu_signer(verifier):
    """signer() for make_txn_stream backed by fd_ed25519_hip_sign_dev."""
    import torch
    dev = torch.device("cuda", verifier.device)

    def sign(prvs, pool, msg_off, msg_sz):
        m = prvs.shape[0]
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        d_prv, d_pool = t(prvs), t(pool)
        d_off, d_sz = t(msg_off.view(np.int32)), t(msg_sz.view(np.int32))
        d_pub = torch.empty((m, 32), dtype=torch.uint8, device=dev)
        d_sig = torch.empty((m, 64), dtype=torch.uint8, device=dev)
        verifier.sign_dev(m, d_prv, d_pool, d_off, d_sz, d_pub, d_sig)
        verifier.sync()
        return d_pub.cpu().numpy(), d_sig.cpu().numpy()

    return sign


TXNM_SZ = 80            # sizeof(fd_txn_m_t) (include/fd_verify_hip.h, src/disco/fd_txn_m.h:15-61)
PARSED_CHUNKS = 34      # FD_TPU_PARSED_MTU (2168 B) in 64-B dcache chunks


def txnm_dcache(pool, off, sz, bundle_id=None, seed=1):
    """Lay frags out as the verify tile's in-link dcache does: each frag an
    fd_txn_m_t (80-byte header: payload_sz at 8, block_engine.bundle_id at 24,
    reference_slot / source fields filled with seeded bytes) followed by its
    payload, at the next free 64-byte chunk (fd_dcache_compact_next).
    Returns (region uint8, chunk uint32[n], frag_sz uint16[n])."""
    n = off.size
    fsz = TXNM_SZ + sz.astype(np.int64)
    nchunk = (fsz + 63) // 64
    chunk = np.concatenate([[0], np.cumsum(nchunk)[:-1]]).astype(np.int64)
    region = np.zeros(int(64 * (chunk[-1] + nchunk[-1])) + 64 if n else 64, np.uint8)
    hdr = np.random.default_rng(seed).integers(0, 256, (n, TXNM_SZ), dtype=np.uint8)
    hdr[:, 8:10] = sz.astype(np.uint16).view(np.uint8).reshape(n, 2)
    hdr[:, 10:12] = 0
    hdr[:, 24:32] = (np.zeros(n, np.uint64) if bundle_id is None else
                     np.asarray(bundle_id, np.uint64)).view(np.uint8).reshape(n, 8)
    base = 64 * chunk
    region[base[:, None] + np.arange(TXNM_SZ)] = hdr
    for j in range(n):
        b = int(base[j]) + TXNM_SZ
        region[b:b + int(sz[j])] = pool[int(off[j]):int(off[j]) + int(sz[j])]
    return region, chunk.astype(np.uint32), fsz.astype(np.uint16)
