"""Synthetic verify workloads (BASELINE.json configs C1-C5), repo-owned.

The validity mix follows SURVEY.md 8(d) (config 2): per signature a seeded
roll picks one of
  10% single random bit flip in the 512-bit signature
   2% S += L                      (S >= L, rejected by fd_curve25519_scalar_validate)
   2% A = one of the 8 small-order encodings   (fd_curve25519.h:91-98)
   2% R = one of the 8 small-order encodings
   2% non-canonical A: y in [p, p+18], sign bit kept
   2% non-canonical R: y in [p, p+18], sign bit kept
   1% public-key bit flip
  79% untouched (valid)
"""
import numpy as np

P_INT = 2**255 - 19
L_INT = 2**252 + 27742317777372353535851937790883648493

SMALL_ORDER_ENCODINGS = [bytes.fromhex(h) for h in (
    "0100000000000000000000000000000000000000000000000000000000000000",
    "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "0000000000000000000000000000000000000000000000000000000000000000",
    "0000000000000000000000000000000000000000000000000000000000000080",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc85",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac03fa",
)]

KIND_VALID, KIND_SIGFLIP, KIND_S_GE_L, KIND_A_SMALL, KIND_R_SMALL, KIND_A_NONCANON, KIND_R_NONCANON, KIND_PUBFLIP = range(8)
_EDGES = np.array([0.10, 0.12, 0.14, 0.16, 0.18, 0.20, 0.21])
_KIND_OF_BIN = np.array([KIND_SIGFLIP, KIND_S_GE_L, KIND_A_SMALL, KIND_R_SMALL, KIND_A_NONCANON,
                         KIND_R_NONCANON, KIND_PUBFLIP, KIND_VALID], np.uint8)


def _noncanon(orig32, k):
    y = P_INT + int(k)                                   # in [p, p+18] < 2^255
    b = bytearray(y.to_bytes(32, "little"))
    b[31] |= orig32[31] & 0x80                            # keep the sign bit
    return np.frombuffer(bytes(b), np.uint8)


def c2_mutate(sigs, pubs, rng):
    """Mutate (n,64) sigs and (n,32) pubs in place; return the per-record kind."""
    n = sigs.shape[0]
    kinds = _KIND_OF_BIN[np.searchsorted(_EDGES, rng.random(n), side="right")]
    idx = np.nonzero(kinds == KIND_SIGFLIP)[0]
    bits = rng.integers(0, 512, size=idx.size)
    sigs[idx, bits >> 3] ^= (1 << (bits & 7)).astype(np.uint8)
    for i in np.nonzero(kinds == KIND_S_GE_L)[0]:
        s = int.from_bytes(sigs[i, 32:].tobytes(), "little") + L_INT
        sigs[i, 32:] = np.frombuffer(s.to_bytes(32, "little"), np.uint8)
    so = np.frombuffer(b"".join(SMALL_ORDER_ENCODINGS), np.uint8).reshape(8, 32)
    idx = np.nonzero(kinds == KIND_A_SMALL)[0]; pubs[idx] = so[rng.integers(0, 8, idx.size)]
    idx = np.nonzero(kinds == KIND_R_SMALL)[0]; sigs[idx, :32] = so[rng.integers(0, 8, idx.size)]
    for i in np.nonzero(kinds == KIND_A_NONCANON)[0]:
        pubs[i] = _noncanon(pubs[i], rng.integers(0, 19))
    for i in np.nonzero(kinds == KIND_R_NONCANON)[0]:
        sigs[i, :32] = _noncanon(sigs[i, :32], rng.integers(0, 19))
    idx = np.nonzero(kinds == KIND_PUBFLIP)[0]
    bits = rng.integers(0, 256, size=idx.size)
    pubs[idx, bits >> 3] ^= (1 << (bits & 7)).astype(np.uint8)
    return kinds


class Batch:
    """A verify batch resident in HBM (torch tensors on one device)."""

    def __init__(self, dev, sigs, pubs, pool, msg_off, msg_sz, kinds=None):
        self.dev, self.sigs, self.pubs, self.pool = dev, sigs, pubs, pool
        self.msg_off, self.msg_sz, self.kinds = msg_off, msg_sz, kinds

    @property
    def n(self):
        return self.sigs.shape[0]


def make_batch_gpu(verifier, n, msg_sz=64, seed=0x5eed0001, mix="c1", shared_msg=False):
    """Config-1 style batch: n random keypairs, one random msg_sz-byte message
    per signature (or one shared message: config 3), signed on the GPU by the
    engine's own signer (fd_ed25519_hip_sign_dev).  mix="c2" applies the C2
    mutation model on the device afterwards (c2_mutate_torch)."""
    import torch
    dev = torch.device("cuda", verifier.device)
    rng = np.random.default_rng(seed)
    prvs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    if shared_msg:
        pool = np.concatenate([rng.integers(0, 256, size=msg_sz, dtype=np.uint8), np.zeros(16, np.uint8)])
        moff = np.zeros(n, np.uint32)
    else:
        pool = np.concatenate([rng.integers(0, 256, size=n * msg_sz, dtype=np.uint8), np.zeros(16, np.uint8)])
        moff = (np.arange(n, dtype=np.uint64) * msg_sz).astype(np.uint32)
    msz = np.full(n, msg_sz, np.uint32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_prv, d_pool = t(prvs), t(pool)
    d_off, d_sz = t(moff.view(np.int32)), t(msz.view(np.int32))
    d_pub = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    verifier.sign_dev(n, d_prv, d_pool, d_off, d_sz, d_pub, d_sig)
    verifier.sync()
    kinds = None
    if mix == "c2":
        kinds = c2_mutate_torch(d_sig, d_pub, seed ^ 0xc2)
    return Batch(dev, d_sig, d_pub, d_pool, d_off, d_sz, kinds)


GLOBAL_BLOCK = 1 << 20


def range_inputs(lo, hi, msg_sz=64, seed=0x5eed0005, block=GLOBAL_BLOCK):
    """Host inputs of records [lo, hi) of a global seeded set (config 5):
    the set is cut into blocks of `block` records, block b drawn from
    default_rng([seed, b]) (private keys, then its messages), so any range --
    one rank's shard or the whole set -- is the same records.  Returns
    (prvs (hi-lo, 32) u8, pool u8 with 16 zero bytes of tail, moff, msz)."""
    b0, b1 = lo // block, (hi + block - 1) // block
    prvs, pool = [], []
    for b in range(b0, b1):
        rng = np.random.default_rng([seed, b])
        p = rng.integers(0, 256, size=(block, 32), dtype=np.uint8)
        m = rng.integers(0, 256, size=block * msg_sz, dtype=np.uint8)
        s0, s1 = max(lo, b * block) - b * block, min(hi, (b + 1) * block) - b * block
        prvs.append(p[s0:s1])
        pool.append(m[s0 * msg_sz:s1 * msg_sz])
    n = hi - lo
    pool = np.concatenate(pool + [np.zeros(16, np.uint8)])
    moff = (np.arange(n, dtype=np.uint64) * msg_sz).astype(np.uint32)
    return np.concatenate(prvs), pool, moff, np.full(n, msg_sz, np.uint32)


def make_batch_gpu_range(verifier, lo, hi, msg_sz=64, seed=0x5eed0005, mix="c2", block=GLOBAL_BLOCK):
    """Records [lo, hi) of the global seeded set (range_inputs), signed on
    the GPU; mix="c2" mutates each block with its own seed, so the verdicts
    of a range equal that range of a whole-set pass (bench.py config 5: each
    rank generates and verifies only its shard)."""
    import torch
    dev = torch.device("cuda", verifier.device)
    prvs, pool, moff, msz = range_inputs(lo, hi, msg_sz, seed, block)
    n = hi - lo
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_pool, d_off, d_sz = t(pool), t(moff.view(np.int32)), t(msz.view(np.int32))
    d_pub = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    verifier.sign_dev(n, t(prvs), d_pool, d_off, d_sz, d_pub, d_sig)
    verifier.sync()
    kinds = None
    if mix == "c2":
        kinds = torch.empty(n, dtype=torch.uint8, device=dev)
        for b in range(lo // block, (hi + block - 1) // block):
            # mutate whole blocks (a block's draws do not depend on the range)
            s0, s1 = max(lo, b * block), min(hi, (b + 1) * block)
            if s0 == b * block and s1 == (b + 1) * block:
                kinds[s0 - lo:s1 - lo] = c2_mutate_torch(d_sig[s0 - lo:s1 - lo], d_pub[s0 - lo:s1 - lo],
                                                         ((seed ^ 0xc2) & 0xffffffff) * 4096 + b)
            else:
                raise ValueError("make_batch_gpu_range with mix='c2' needs block-aligned ranges")
    return Batch(dev, d_sig, d_pub, d_pool, d_off, d_sz, kinds)


def c2_mutate_torch(sigs, pubs, seed):
    """The C2 mutation model on device tensors ((n,64) / (n,32) uint8), in
    place, for batches too large for the host loop; same distribution as
    c2_mutate (different draws).  Returns the per-record kind (uint8)."""
    import torch
    dev = sigs.device
    n = sigs.shape[0]
    g = torch.Generator(device=dev)
    g.manual_seed(int(seed))
    roll = torch.rand(n, generator=g, device=dev)
    edges = torch.tensor(_EDGES, device=dev, dtype=roll.dtype)
    kinds = torch.tensor(_KIND_OF_BIN, device=dev)[torch.bucketize(roll, edges, right=True)]

    def flip(buf, nbits, mask_kind):
        idx = torch.nonzero(kinds == mask_kind).flatten()
        if idx.numel():
            bit = torch.randint(0, nbits, (idx.numel(),), generator=g, device=dev)
            buf[idx, bit >> 3] ^= (1 << (bit & 7)).to(torch.uint8)

    flip(sigs, 512, KIND_SIGFLIP)
    flip(pubs, 256, KIND_PUBFLIP)
    # S += L on 8 little-endian 32-bit limbs (S < L, so no overflow of 2^256)
    idx = torch.nonzero(kinds == KIND_S_GE_L).flatten()
    if idx.numel():
        s = sigs[idx, 32:].to(torch.int64).view(-1, 8, 4)
        limbs = s[..., 0] | (s[..., 1] << 8) | (s[..., 2] << 16) | (s[..., 3] << 24)
        lw = torch.tensor([(L_INT >> (32 * i)) & 0xffffffff for i in range(8)], device=dev, dtype=torch.int64)
        carry = torch.zeros(idx.numel(), dtype=torch.int64, device=dev)
        for i in range(8):
            t = limbs[:, i] + lw[i] + carry
            limbs[:, i] = t & 0xffffffff
            carry = t >> 32
        out = torch.stack([(limbs >> (8 * b)) & 0xff for b in range(4)], dim=-1).reshape(-1, 32)
        sigs[idx, 32:] = out.to(torch.uint8)
    so = torch.tensor(list(b"".join(SMALL_ORDER_ENCODINGS)), dtype=torch.uint8, device=dev).view(8, 32)
    idx = torch.nonzero(kinds == KIND_A_SMALL).flatten()
    if idx.numel():
        pubs[idx] = so[torch.randint(0, 8, (idx.numel(),), generator=g, device=dev)]
    idx = torch.nonzero(kinds == KIND_R_SMALL).flatten()
    if idx.numel():
        sigs[idx, :32] = so[torch.randint(0, 8, (idx.numel(),), generator=g, device=dev)]

    def noncanon(buf, cols):
        # y = p + k (k in [0,18]) < 2^255: byte0 = 0xed + k, bytes 1..30 = 0xff, byte31 = 0x7f | sign
        k = torch.randint(0, 19, (cols.numel(),), generator=g, device=dev)
        sign = buf[cols, 31] & 0x80
        enc = torch.full((cols.numel(), 32), 0xff, dtype=torch.uint8, device=dev)
        enc[:, 0] = (0xed + k).to(torch.uint8)
        enc[:, 31] = 0x7f | sign
        buf[cols, :32] = enc

    idx = torch.nonzero(kinds == KIND_A_NONCANON).flatten()
    if idx.numel():
        noncanon(pubs, idx)
    idx = torch.nonzero(kinds == KIND_R_NONCANON).flatten()
    if idx.numel():
        noncanon(sigs, idx)
    return kinds
