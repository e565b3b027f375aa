"""GPU: the sharded (N>1) verify path with real kernels.

1. Two fresh rank processes (tests/multi_rank_worker.py, gloo group, one
   verify context each on GPU 0) verify their shard_bounds halves of one
   2^23-signature C2-mix batch and all-gather the verdict bitmap; it must
   equal a single-process whole-batch pass, whose codes must equal the CPU
   oracle on an 8K sample (BASELINE configs[4]).
2. bench.py's own N>1 code (torch.distributed.run, max-over-ranks time,
   all-reduced signature count, C5 strong-scaling shards) at world size 2,
   rehearsed with --dist-backend gloo because both ranks share the box's one
   GPU (RCCL refuses two ranks on one device).

The ranks are started as child processes of this (GPU-initialised) test
process with subprocess, never by exec.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_two_ranks_shard_and_gather(tmp_path):
    n, world = 1 << 23, 2
    port = _free_port()
    procs, outs = [], []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out = tmp_path / f"rank{r}.json"
        outs.append(out)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "multi_rank_worker.py"), str(n), str(out)],
                                      env=env, cwd=REPO))
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=240))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert rcs == [0] * world, rcs
    res = [json.load(open(o)) for o in outs]
    assert res[0]["lo"] == 0 and res[-1]["hi"] == n and res[0]["hi"] == res[1]["lo"]
    r0 = res[0]
    assert r0["bitmap_equal"], r0
    assert r0["bitmap_is_codes"] and r0["codes_set"], r0
    assert r0["oracle_sample_equal"], r0
    assert 0.75 < r0["accept"] < 0.83, r0


@pytest.mark.gpu
def test_bench_world2_default_line_gloo():
    """The default bench line (C2 leg + the c4 sub-object) at world 2, as the
    driver's scaling runs launch it (gloo here: two ranks on one GPU):
    one JSON line, both legs' values present, the c4 leg's signatures
    summed over the ranks."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
           "--sigs", str(1 << 18), "--txns", str(1 << 16), "--steps", "2", "--warmup", "1",
           "--c4-pcie-steps", "1", "--dist-backend", "gloo", "--no-cpu-baseline", "--no-tile"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and "tile" not in d
    assert d["c4"]["value"] > 0 and d["c4"]["config"]["frags_per_gpu"] == 1 << 16


@pytest.mark.gpu
def test_bench_world2_c5_gloo(tmp_path):
    """bench.py's N>1 path at world 2 (gloo: RCCL refuses two ranks on one
    GPU): the JSON line carries the CPU baseline, and the two ranks'
    verdicts -- each rank generates and verifies only its shard of the one
    global C5 set -- equal a one-process pass over the whole set."""
    port = _free_port()
    import numpy as np
    import torch

    import bench
    from firedancer_amd import Verifier
    from firedancer_amd.workload import make_batch_gpu_range
    prefix = str(tmp_path / "codes")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
           "--config", "c5", "--sigs", str(1 << 21), "--steps", "2", "--warmup", "1",
           "--dist-backend", "gloo", "--cpu-seconds", "1", "--dump-codes", prefix]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["config"]["config_id"] == "c5"
    assert d["value"] > 0 and d["steps"] == 2
    assert str(1 << 22) in d["config"]["workload"]          # n_all all-reduced over both ranks
    cpu = d["cpu_baseline"]
    assert cpu and cpu["value"] > 0 and cpu["kind"] == "reference" and cpu.get("codes_match") is True, cpu
    total = 1 << 22
    got = np.concatenate([np.load(f"{prefix}.{rk}.npy") for rk in range(2)])
    for rk in range(2):
        t, lo, hi = bench.c5_shard(1 << 21, rk, 2)
        assert t == total and np.load(f"{prefix}.{rk}.npy").size == hi - lo
    v = Verifier(device=0, chunk_sigs=1 << 20)
    b = make_batch_gpu_range(v, 0, total)
    codes = torch.zeros(total, dtype=torch.int8, device=b.dev)
    v.verify_dev(total, b.sigs, b.pubs, b.pool, b.msg_off, b.msg_sz, codes)
    v.sync()
    whole = codes.cpu().numpy()
    v.close()
    assert np.array_equal(got, whole)
    assert 0.75 < float((whole == 0).mean()) < 0.83


@pytest.mark.gpu
def test_c5_full_size_sharded_on_one_gpu():
    """BASELINE configs[4] at its full size: 2^26 C2-mix signatures, cut by
    bench's c5_shard for world 8 and verified shard by shard on 8 contexts of
    this one GPU (what 8 ranks do on 8 GPUs); the concatenated shard bitmaps
    equal the codes, every mutation class lands in its rejection class, the
    accept rate is the C2 mix's, and a 4K sample is bit-exact against the
    oracle."""
    import numpy as np
    import torch

    import bench
    import oracle_lib as O
    from firedancer_amd import Verifier
    from firedancer_amd import workload as W
    from firedancer_amd.ed25519 import CTX_STREAM
    n, world = 1 << 26, 8
    dev = torch.device("cuda", 0)
    gen = Verifier(device=0, chunk_sigs=1 << 20)
    b = W.make_batch_gpu_range(gen, 0, n)                  # the global set bench.py's C5 ranks shard
    codes = torch.full((n,), 9, dtype=torch.int8, device=dev)
    bm = torch.zeros(n // 64, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    ctxs = []
    for r in range(world):
        total, lo, hi = bench.c5_shard(None, r, world)
        assert total == n
        v = Verifier(device=0, chunk_sigs=1 << 20)
        ctxs.append(v)
        v.verify_dev(hi - lo, b.sigs[lo:hi], b.pubs[lo:hi], b.pool, b.msg_off[lo:hi], b.msg_sz[lo:hi],
                     codes[lo:hi], bm[lo // 64:hi // 64], stream=CTX_STREAM)
    for v in ctxs:
        v.sync()
    c = codes.cpu().numpy()
    kinds = b.kinds.cpu().numpy()
    assert np.isin(c, (0, -1, -2, -3)).all()
    bits = np.unpackbits(bm.cpu().numpy().view(np.uint8), bitorder="little").astype(bool)
    assert np.array_equal(bits, c == 0)
    assert (c[kinds == W.KIND_VALID] == 0).all()
    assert (c[kinds == W.KIND_S_GE_L] == -1).all()
    assert (c[kinds == W.KIND_A_SMALL] == -2).all()
    assert (c[kinds == W.KIND_R_SMALL] == -1).all()
    assert (c[kinds == W.KIND_SIGFLIP] != 0).all() and (c[kinds == W.KIND_PUBFLIP] != 0).all()
    assert 0.77 < float((c == 0).mean()) < 0.81
    idx = np.sort(np.random.default_rng(26).choice(n, 4096, replace=False))
    ti = torch.from_numpy(idx).to(dev)
    msgs = b.pool[:n * 64].view(n, 64)[ti].cpu().numpy()                  # message i = pool[64i, +64)
    pool = np.concatenate([msgs.reshape(-1), np.zeros(16, np.uint8)])
    exp = O.verify_many(b.sigs[ti].cpu().numpy(), b.pubs[ti].cpu().numpy(), pool,
                        (np.arange(idx.size) * 64).astype(np.uint32), np.full(idx.size, 64, np.uint32))
    assert np.array_equal(c[idx], exp)
    for v in ctxs + [gen]:
        v.close()
