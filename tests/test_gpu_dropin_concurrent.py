"""GPU: concurrent callers of the drop-in API.

The reference's fd_ed25519_verify / _batch_single_msg are re-entrant with no
global mutable state (src/ballet/ed25519/fd_ed25519.h:89-94), and replay
calls them per transaction from many threads
(src/flamenco/runtime/fd_executor.c:1608-1617).  The engine combines
concurrent calls into shared launches (fd_ed25519_hip.hip, the drop-in
staging ring); these tests drive it from many host threads (ctypes releases
the GIL for the whole C call) and check every result against the
reference's own verdicts (tests/golden/ref_scale_groups.npz) and the
oracle."""
import os
import threading
import time

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _groups():
    d = np.load(os.path.join(GOLDEN, "ref_scale_groups.npz"))
    return {k: d[k] for k in d.files}


def _run_threads(nthreads, fn):
    errs = []

    def wrap(t):
        try:
            fn(t)
        except BaseException as e:              # noqa: BLE001 -- reported below
            errs.append(e)
    ths = [threading.Thread(target=wrap, args=(t,)) for t in range(nthreads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    if errs:
        raise errs[0]


def test_dropin_init_entry():
    from firedancer_amd.ed25519 import fd_ed25519_hip_dropin_init
    assert fd_ed25519_hip_dropin_init(0) == 0
    assert fd_ed25519_hip_dropin_init(0) == 0           # idempotent
    assert fd_ed25519_hip_dropin_init(7) == -1          # exists on another device


def test_concurrent_batch_single_msg_equals_reference():
    """16 threads share the fixture's 4096 batch_single_msg groups (AVX-512
    codes) and a mixed stream of single verifies; every call's code must be
    the reference's, and calls must have been combined."""
    from firedancer_amd import fd_ed25519_verify, fd_ed25519_verify_batch_single_msg
    from firedancer_amd.ed25519 import dropin_stats
    g = _groups()
    sigs, pubs, pool = g["sigs"], g["pubs"], g["pool"]
    first, cnt, moff, msz, exp = g["first"], g["cnt"], g["msg_off"], g["msg_sz"], g["gcode_avx512"]
    nrec, ng, T = sigs.shape[0], first.size, 16
    got = np.full(ng, 9, np.int8)
    single_exp = {}

    def worker(t):
        for gi in range(t, ng, T):
            f, c = int(first[gi]), int(cnt[gi])
            k = min(max(c, 1), nrec - f)
            m = pool[int(moff[f]):int(moff[f]) + int(msz[f])].tobytes()
            got[gi] = fd_ed25519_verify_batch_single_msg(m, sigs[f:f + k].tobytes(), pubs[f:f + k].tobytes(), c)
            if gi % 7 == 0:                              # interleave single verifies of the group's first record
                r = fd_ed25519_verify(m, sigs[f].tobytes(), pubs[f].tobytes())
                single_exp[gi] = (r, O.verify(m, sigs[f].tobytes(), pubs[f].tobytes()))

    before = dropin_stats()
    _run_threads(T, worker)
    after = dropin_stats()
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, [(int(i), int(got[i]), int(exp[i])) for i in bad[:10]]
    assert all(a == b for a, b in single_exp.values())
    launches, calls = after[0] - before[0], after[1] - before[1]
    real = int(((cnt >= 1) & (cnt <= 16)).sum())           # 0 / 17 return ERR_SIG before staging
    assert calls == real + len(single_exp), (calls, real, len(single_exp))
    assert launches < calls, (launches, calls)          # concurrent calls shared launches
    print(f"concurrent drop-in: {calls} calls in {launches} launches ({calls / launches:.2f} per launch)")


def test_concurrent_throughput_12_sig_calls():
    """16 threads, each calling batch_single_msg with 12 valid signatures
    over its own 64-byte message in a loop for ~3 s: aggregate signatures/s
    and per-call latency are printed (measured, not asserted beyond
    correctness: every call must return SUCCESS)."""
    from firedancer_amd import fd_ed25519_verify_batch_single_msg
    from firedancer_amd.ed25519 import dropin_stats
    T, K = 16, 12
    rng = np.random.default_rng(0x16)
    msgs = rng.integers(0, 256, (T, 64), dtype=np.uint8)
    prvs = rng.integers(0, 256, (T * K, 32), dtype=np.uint8)
    pool = msgs.reshape(-1)
    moff = np.repeat(np.arange(T, dtype=np.uint32) * 64, K)
    msz = np.full(T * K, 64, np.uint32)
    pubs, sigs = O.sign_many(prvs, pool, moff, msz)
    lat = [[] for _ in range(T)]
    bad = []
    stop = time.monotonic() + 3.0

    def worker(t):
        m, s, p = msgs[t].tobytes(), sigs[t * K:(t + 1) * K].tobytes(), pubs[t * K:(t + 1) * K].tobytes()
        while time.monotonic() < stop:
            t0 = time.perf_counter()
            r = fd_ed25519_verify_batch_single_msg(m, s, p, K)
            lat[t].append(time.perf_counter() - t0)
            if r != 0:
                bad.append(r)

    fd_ed25519_verify_batch_single_msg(msgs[0].tobytes(), sigs[:K].tobytes(), pubs[:K].tobytes(), K)   # warm
    before = dropin_stats()
    t0 = time.monotonic()
    _run_threads(T, worker)
    dt = time.monotonic() - t0
    after = dropin_stats()
    assert not bad, bad[:5]
    calls = sum(len(x) for x in lat)
    allat = np.array(sum(lat, [])) * 1e6
    launches = after[0] - before[0]
    print(f"16 threads x batch_single_msg(12): {calls * K / dt / 1e6:.3f} M sigs/s, {calls / dt:.0f} calls/s, "
          f"p50 {np.percentile(allat, 50):.0f} us, p99 {np.percentile(allat, 99):.0f} us, "
          f"{calls / max(launches, 1):.1f} calls per launch")
    assert calls > 0


HARNESS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "dropin_threads")


def _harness_input(path, T, K, msg_sz, seed):
    rng = np.random.default_rng(seed)
    msgs = rng.integers(0, 256, (T, msg_sz), dtype=np.uint8)
    prvs = rng.integers(0, 256, (T * K, 32), dtype=np.uint8)
    pool = msgs.reshape(-1)
    moff = np.repeat(np.arange(T, dtype=np.uint32) * msg_sz, K)
    msz = np.full(T * K, msg_sz, np.uint32)
    pubs, sigs = O.sign_many(prvs, pool, moff, msz)
    with open(path, "wb") as f:
        f.write(np.array([T, K, msg_sz, 0], np.uint32).tobytes())
        for t in range(T):
            f.write(msgs[t].tobytes())
            f.write(np.ascontiguousarray(sigs[t * K:(t + 1) * K]).tobytes())
            f.write(np.ascontiguousarray(pubs[t * K:(t + 1) * K]).tobytes())


def test_concurrent_c_callers(tmp_path):
    """tools/dropin_threads (built by build(); a missing binary fails, it is
    not skipped): 1, 16 and 64 C threads each calling batch_single_msg with
    12 valid signatures over its own 64-byte message for 2 s.  Every call must
    return SUCCESS; aggregate signatures/s and latency percentiles are
    printed (the measurement of record, no ctypes/GIL in the loop)."""
    import json
    import subprocess
    assert os.path.exists(HARNESS), "tools/dropin_threads missing: run __graft_entry__.build()"
    inp = str(tmp_path / "calls.bin")
    _harness_input(inp, 64, 12, 64, 0x1612)
    out = {}
    for threads in (1, 16, 64):
        r = subprocess.run([HARNESS, inp, "2", str(threads)], capture_output=True, text=True, timeout=90)
        assert r.returncode == 0, (threads, r.stdout, r.stderr[-2000:])
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["bad"] == 0 and d["calls"] > 0, d
        out[threads] = d
        print(f"C callers {threads:3d} x batch_single_msg(12): {d['sigs_per_s'] / 1e6:.3f} M sigs/s, "
              f"p50 {d['p50_us']:.0f} us, p99 {d['p99_us']:.0f} us, {d['calls_per_launch']:.2f} calls/launch")
    with open(str(tmp_path / "summary.json"), "w") as f:
        json.dump(out, f)
    dst = os.environ.get("FD_DROPIN_SUMMARY")
    if dst:
        with open(dst, "w") as f:
            json.dump(out, f, indent=1)


def test_concurrent_mixed_sizes_and_long_messages():
    """12 threads mixing single verifies and batch_single_msg calls of 1..16
    signatures over messages of 0 B .. 200 KB (past a staging block's initial
    64-KB message area, so blocks grow while other batch slots run), with
    corrupted signatures mixed in: every code equals the oracle's."""
    from firedancer_amd import fd_ed25519_verify, fd_ed25519_verify_batch_single_msg
    rng = np.random.default_rng(0x5107)
    T, CALLS = 12, 12
    jobs = []
    for t in range(T):
        for c in range(CALLS):
            sz = int(rng.choice([0, 1, 63, 200, 1232, 5000, 70000, 200000]))
            k = int(rng.integers(1, 17))
            msg = rng.integers(0, 256, sz, dtype=np.uint8)
            prvs = rng.integers(0, 256, (k, 32), dtype=np.uint8)
            pubs, sigs = O.sign_many(prvs, msg, np.zeros(k, np.uint32), np.full(k, sz, np.uint32))
            sigs = sigs.copy()
            if rng.random() < 0.3:                          # corrupt one signature's R or S
                j = int(rng.integers(0, k)); sigs[j, int(rng.integers(0, 64))] ^= 0x40
            jobs.append((t, msg.tobytes(), sigs, pubs, k))
    got = {}

    def worker(t):
        for ji, (tt, m, s, p, k) in enumerate(jobs):
            if tt != t:
                continue
            if k == 1 and ji % 2 == 0:
                got[ji] = fd_ed25519_verify(m, s[0].tobytes(), p[0].tobytes())
            else:
                got[ji] = fd_ed25519_verify_batch_single_msg(m, s.tobytes(), p.tobytes(), k)

    _run_threads(T, worker)
    for ji, (t, m, s, p, k) in enumerate(jobs):
        if k == 1 and ji % 2 == 0:
            exp = O.verify(m, s[0].tobytes(), p[0].tobytes())
        else:
            exp = O.verify_batch_single_msg(m, s.tobytes(), p.tobytes(), k)
        assert got[ji] == exp, (ji, len(m), k, got[ji], exp)
