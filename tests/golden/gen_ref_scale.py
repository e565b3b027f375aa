#!/usr/bin/env python3
"""Generate the reference-verdict fixtures at scale (committed under tests/golden/).

Runs ONLY in the build container.  Inputs are signed by the reference's own
fd_ed25519_sign (oracle/_ref/libfdref_avx512.so, compiled from
/root/reference sources by oracle/Makefile) and the verdicts come from the
reference's own fd_ed25519_verify / fd_ed25519_verify_batch_single_msg
(oracle/_ref/ref_cpu_bench_{avx512,ref}: the AVX-512 IFMA backend and the
portable fiat-crypto backend, src/ballet/ed25519/fd_ed25519_user.c:135-310).
The GPU box never runs the reference: tests/test_gpu_ref_fixture.py compares
the engine against these stored codes.

ref_scale_records.npz -- 2^16 single verifies (user.c:135-230)
  messages are windows of a shared random pool (0..1232 bytes, and 64
  messages of 1233..16383); every record has its own key; the C2 mutation model
  (firedancer_amd/workload.py) then the ten extra classes of
  tests/fdgen.extra_mutations on the still-valid records (a record whose
  message gets a bit flip first receives a private copy of its window).
  Arrays: sigs (n,64) pubs (n,32) msg_off msg_sz pool kinds extra,
  code_avx512 code_ref.
ref_scale_groups.npz -- 2^12 batch_single_msg calls (user.c:232-310)
  group g = records [first[g], first[g]+cnt[g]) over one per-group message
  window, cnt in 1..16 plus a few 0 and 17 (ERR_SIG, user.c:238-241; a 17
  reads the next group's first record, as the reference would); sparse C2
  mutations (4% of the records) and message flips on 2% of the groups (most
  groups verify; every code occurs).  Arrays: sigs pubs msg_off msg_sz (per
  record, the group's message) pool first cnt, gcode_avx512 gcode_ref.

usage: python tests/golden/gen_ref_scale.py   (after `make -C oracle all`)
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "tests"))
from gen_golden import RefLib  # noqa: E402
from fdgen import c2_mutate, extra_mutations, msg_sizes  # noqa: E402

REF_DIR = os.path.join(REPO, "oracle", "_ref")
N_REC = 1 << 16
N_GRP = 1 << 12
POOL = 1 << 16                  # shared window pool (plus the long-message region)


def write_fdv1(path, sigs, pubs, pool, moff, msz, bfirst=None, bcnt=None):
    """Input file of oracle/ref_cpu_bench.c ("FDV1")."""
    nb = 0 if bfirst is None else len(bfirst)
    with open(path, "wb") as f:
        f.write(b"FDV1")
        f.write(np.array([sigs.shape[0], pool.size, nb], np.uint64).tobytes())
        for a in (sigs, pubs, moff.astype(np.uint32), msz.astype(np.uint32), pool):
            f.write(np.ascontiguousarray(a).tobytes())
        if nb:
            f.write(np.asarray(bfirst, np.uint32).tobytes())
            f.write(np.asarray(bcnt, np.uint8).tobytes())


def run_ref(backend, *arrays, **kw):
    exe = os.path.join(REF_DIR, f"ref_cpu_bench_{backend}")
    with tempfile.TemporaryDirectory() as d:
        inp, out = os.path.join(d, "in.bin"), os.path.join(d, "codes.bin")
        write_fdv1(inp, *arrays, **kw)
        subprocess.run([exe, inp, str(os.cpu_count() or 1), out], check=True, stdout=subprocess.DEVNULL)
        return np.fromfile(out, np.int8)


def windows(rng, sizes, pool_sz, long_base):
    """Offsets of message windows: short ones anywhere in [0, pool_sz - sz],
    long ones (> 1232 B) consecutive from long_base."""
    off = np.zeros(sizes.size, np.uint32)
    cur = long_base
    for i, s in enumerate(sizes):
        if s > 1232:
            off[i] = cur
            cur += int(s)
        else:
            off[i] = rng.integers(0, pool_sz - int(s) + 1)
    return off, cur


def sign_all(ref, prvs, pool, moff, msz):
    n = prvs.shape[0]
    sigs = np.zeros((n, 64), np.uint8)
    pubs = np.zeros((n, 32), np.uint8)
    for i in range(n):
        prv = prvs[i].tobytes()
        pk = ref.pub_from_prv(prv)
        pubs[i] = np.frombuffer(pk, np.uint8)
        m = pool[moff[i]:moff[i] + msz[i]].tobytes()
        sigs[i] = np.frombuffer(ref.sign(m, pk, prv), np.uint8)
    return sigs, pubs


def gen_records(ref):
    rng = np.random.default_rng(0x5ca1e001)
    msz = msg_sizes(rng, N_REC, hi=16383)
    big = np.nonzero(msz > 1232)[0]                     # keep 64 long messages (fixture size)
    msz[big[64:]] = rng.integers(0, 1233, big.size - 64)
    long_sz = int(msz[msz > 1232].astype(np.int64).sum())
    pool = rng.integers(0, 256, POOL + long_sz + 64, dtype=np.uint8)
    moff, _ = windows(rng, msz, POOL, POOL)
    prvs = rng.integers(0, 256, (N_REC, 32), dtype=np.uint8)
    sigs, pubs = sign_all(ref, prvs, pool, moff, msz)
    kinds = c2_mutate(sigs, pubs, rng)
    # a bit flip must hit only its own record: give every record that may be
    # flipped a private copy of its window first (class 4 is drawn inside
    # extra_mutations, so copy for all still-valid records' candidates)
    valid = kinds == 0
    rng_x = np.random.default_rng(0x5ca1e002)
    probe = rng_x.permutation(np.nonzero(valid)[0])
    k = probe.size // 40
    flip = probe[4 * k:5 * k]                          # the records extra_mutations' class 4 will pick
    extra_pool = [pool]
    cur = pool.size
    for i in flip:
        s = int(msz[i])
        extra_pool.append(pool[moff[i]:moff[i] + s].copy())
        moff[i] = cur
        cur += s
    extra_pool.append(np.zeros(64, np.uint8))
    pool = np.concatenate(extra_pool)
    cls = extra_mutations(np.random.default_rng(0x5ca1e002), sigs, pubs, pool, moff, msz, valid)
    assert np.array_equal(np.sort(cls[4]), np.sort(flip))
    extra = np.zeros(N_REC, np.int8)
    for c, ix in enumerate(cls):
        extra[ix] = c + 1
    ca = run_ref("avx512", sigs, pubs, pool, moff, msz)
    cr = run_ref("ref", sigs, pubs, pool, moff, msz)
    assert np.array_equal(ca == 0, cr == 0)
    np.savez_compressed(os.path.join(HERE, "ref_scale_records.npz"), sigs=sigs, pubs=pubs, msg_off=moff,
                        msg_sz=msz, pool=pool, kinds=kinds, extra=extra, code_avx512=ca, code_ref=cr)
    print("records", N_REC, "pool", pool.size, "avx512", {int(c): int((ca == c).sum()) for c in np.unique(ca)},
          "ref", {int(c): int((cr == c).sum()) for c in np.unique(cr)})


def gen_groups(ref):
    rng = np.random.default_rng(0x5ca1e003)
    cnt = rng.integers(1, 17, N_GRP).astype(np.uint8)
    odd = rng.permutation(N_GRP - 1)[:48]               # never the last group (a 17 reads one record on)
    cnt[odd[:24]] = 0
    cnt[odd[24:]] = 17
    stored = np.maximum(cnt, 1).astype(np.int64)        # records stored per group (a 17 stores 16 + borrows)
    stored[cnt == 17] = 16
    first = np.concatenate([[0], np.cumsum(stored)[:-1]]).astype(np.uint32)
    n = int(stored.sum())
    gsz = msg_sizes(rng, N_GRP, hi=1232)
    pool = rng.integers(0, 256, POOL + 64, dtype=np.uint8)
    goff, _ = windows(rng, gsz, POOL, POOL)
    grp = np.repeat(np.arange(N_GRP), stored)
    moff, msz = goff[grp].copy(), gsz[grp].copy()
    prvs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    sigs, pubs = sign_all(ref, prvs, pool, moff, msz)
    sub = rng.random(n) < 0.04
    s_sigs, s_pubs = sigs[sub].copy(), pubs[sub].copy()
    c2_mutate(s_sigs, s_pubs, rng)
    sigs[sub], pubs[sub] = s_sigs, s_pubs
    # message flips hit a whole group: private copies of those groups' windows
    flip = rng.choice(N_GRP, N_GRP // 50, replace=False)
    parts, cur = [pool], pool.size
    for g in flip:
        s = int(gsz[g])
        if not s:
            continue
        w = pool[goff[g]:goff[g] + s].copy()
        w[int(rng.integers(0, s))] ^= 0x10
        parts.append(w)
        moff[grp == g] = cur
        cur += s
    parts.append(np.zeros(64, np.uint8))
    pool = np.concatenate(parts)
    ga = run_ref("avx512", sigs, pubs, pool, moff, msz, bfirst=first, bcnt=cnt)
    gr = run_ref("ref", sigs, pubs, pool, moff, msz, bfirst=first, bcnt=cnt)
    assert np.array_equal(ga == 0, gr == 0)
    np.savez_compressed(os.path.join(HERE, "ref_scale_groups.npz"), sigs=sigs, pubs=pubs, msg_off=moff, msg_sz=msz,
                        pool=pool, first=first, cnt=cnt, gcode_avx512=ga, gcode_ref=gr)
    print("groups", N_GRP, "records", n, "avx512", {int(c): int((ga == c).sum()) for c in np.unique(ga)},
          "ref", {int(c): int((gr == c).sum()) for c in np.unique(gr)})


def main():
    ref = RefLib(os.path.join(REF_DIR, "libfdref_avx512.so"))
    gen_records(ref)
    gen_groups(ref)


if __name__ == "__main__":
    main()
