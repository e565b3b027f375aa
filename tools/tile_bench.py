#!/usr/bin/env python3
"""Time the reference's verify tile patched to use the engine (north star's
operating point), in the reference's own stem loop, on one GPU.

For each configuration: one producer process (integration/_build/tile_run
produce: the quic side of the quic_verify link, frags pre-laid in its dcache,
mcache lines published with flow control) and T verify tile processes
(tile_run tile: fd_verify_tile.c + integration/fd_verify_tile_hip.patch,
privileged_init / unprivileged_init / stem_run1), each taking seq % T as the
reference's verify tiles do.  The tiles are processes, not threads, as in the
reference; each has its own HIP context and hardware queues.

value = signatures the tiles' GPU batches verified / (last tile done - first
frag published).  Also reported per configuration: frags/s, per-batch GPU and
host-pass times, outcome counts (parse / verify / dedup failures, published).

The stream is config C4's generator (firedancer_amd/txn_workload.py, GPU
signer), --frags frags.  Binaries per (batch_max, inflight) setting are built
here (integration/Makefile, needs /root/reference) and travel to the GPU box.

usage: python tools/tile_bench.py [--frags N] [--tiles 4,6,8] [--configs b4096i2,b8192i3 ...]
       python tools/tile_bench.py --build          (build the sweep's binaries; CPU side)
Prints one JSON line per run and a final summary line."""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
BUILD = os.path.join(REPO, "integration", "_build")
# (batch_max, inflight, gpu_copy): the patch's FD_VERIFY_HIP_* settings; gpu_copy 0 is the host
# during_frag copy ("h" suffix)
SWEEP = [(b, i, g) for b in (1024, 2048, 4096, 8192) for i in (2, 3, 4) for g in (1, 0)] + \
        [(b, i, 1) for b in (16384, 32768, 65536) for i in (2, 3, 4)] + \
        [(b, i, 1) for b in (16384, 32768, 65536) for i in (6, 8)] + \
        [(131072, i, 1) for i in (2, 3)]                                # range mode: few host cycles per frag


def binary(b, i, g=1):
    return os.path.join(BUILD, f"tile_run_b{b}i{i}" + ("" if g else "h"))


def parse_config(cfg):
    """b<batch_max>i<inflight>[h|r] -> (batch_max, inflight, gpu_copy); h: the host during_frag
    copy, r: range mode (the GPU-copy binary with the quic_verify link unpolled, is_range())"""
    g = 0 if cfg.endswith("h") else 1
    b, i = cfg.rstrip("hr")[1:].split("i")
    return int(b), int(i), g


def is_range(cfg):
    return cfg.endswith("r")


def build():
    for b, i, g in SWEEP:
        v = os.path.basename(binary(b, i, g))[len("tile_run"):]
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "integration"), f"VARIANT={v}",
                               f"DEFS=-DFD_VERIFY_HIP_BATCH_MAX={b}UL -DFD_VERIFY_HIP_INFLIGHT={i}UL "
                               f"-DFD_VERIFY_HIP_RANGE_BATCH_MAX={b}UL "
                               f"-DFD_VERIFY_HIP_GPU_COPY={g}", f"_build/tile_run{v}"])
        print(binary(b, i, g))


def make_stream(n, path, seed=0x5eed0004, depth=4194302):
    import torch  # noqa: F401
    from firedancer_amd import Verifier
    from firedancer_amd.txn_workload import gpu_signer, make_txn_stream
    from tile_io import write_fdt1
    v = Verifier(device=0, chunk_sigs=1 << 20)
    s = make_txn_stream(n, gpu_signer(v), seed=seed)
    v.close()
    write_fdt1(path, s.pool, s.off, s.sz, np.zeros(s.n, np.uint64), 0x7f4a11, depth)
    return s


def run_one(exe, stream, tiles, in_depth, timeout, logdir, walk=False, range_mode=False, prelay=False,
            rocprof=None, hw_queues=None, links=1):
    """One producer and `tiles` tile processes; every process's stderr goes to
    a file in logdir; liveness is checked every second (a tile that dies ends
    the run at once), with a progress line on stderr.  range_mode: the tiles
    read the link by range (TILE_RUN_RANGE, tile_run.c)."""
    shm = f"/dev/shm/fd_tile_bench_{os.getpid()}"
    if os.path.exists(shm):
        os.unlink(shm)
    os.makedirs(logdir, exist_ok=True)
    perr = open(os.path.join(logdir, "producer.err"), "w")
    renv = dict(os.environ, TILE_RUN_RANGE="1") if range_mode else None
    penv = dict(renv or os.environ, TILE_RUN_PRELAY="1") if prelay else renv
    if links != 1:                            # quic_verify links, as with that many quic tiles
        penv = dict(penv or os.environ, TILE_RUN_LINKS=str(links))
    prod = subprocess.Popen([exe, "produce", shm, stream, str(tiles), str(in_depth)], stdout=subprocess.PIPE,
                            stderr=perr, text=True, env=penv)
    procs, terr = [], []
    t0 = time.time()
    try:
        line = prod.stdout.readline()
        if line.strip() != "READY":
            raise RuntimeError(f"producer: {line!r} (see {logdir}/producer.err)")
        for t in range(tiles):
            terr.append(open(os.path.join(logdir, f"tile{t}.err"), "w"))
            env = dict(os.environ, TILE_RUN_WALK="1") if walk else renv
            if hw_queues:                     # HIP hardware queues per tile process (one per in-flight slot)
                env = dict(env or os.environ, GPU_MAX_HW_QUEUES=str(hw_queues))
            cmd = [exe, "tile", shm, str(t)]
            if rocprof:                       # each tile under its own kernel trace (the program itself after --)
                cmd = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", rocprof,
                       "-o", f"tile{t}", "--"] + cmd
            procs.append(subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=terr[-1], env=env))
        last = 0.0
        while prod.poll() is None:
            dead = [(t, p.returncode) for t, p in enumerate(procs) if p.poll() is not None and p.returncode]
            if dead:
                raise RuntimeError(f"tile(s) died: {dead} (see {logdir}/tile*.err)")
            if time.time() - t0 > timeout:
                raise RuntimeError(f"timeout after {timeout} s")
            if time.time() - last >= 10.0:
                print(f"  run: {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
                last = time.time()
            time.sleep(0.2)
        out = prod.stdout.read()
        if prod.returncode:
            raise RuntimeError(f"producer rc {prod.returncode} (see {logdir}/producer.err)")
        for t, p in enumerate(procs):
            p.wait(timeout=60)
            if p.returncode:
                raise RuntimeError(f"tile {t} rc {p.returncode} (see {logdir}/tile{t}.err)")
        return json.loads(out.strip().splitlines()[-1])
    finally:
        for p in procs + [prod]:
            if p.poll() is None:
                p.kill()
                p.wait()
        for f in terr + [perr]:
            f.close()
        if os.path.exists(shm):
            os.unlink(shm)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--frags", type=int, default=1 << 21)
    ap.add_argument("--tiles", default="6")
    ap.add_argument("--configs", default="b4096i2",
                    help="b<batch_max>i<inflight>[h|r], comma-separated (binaries from --build; h: host during_frag "
                         "copy; r: range mode, the quic_verify link unpolled)")
    ap.add_argument("--in-depth", type=int, default=16384,
                    help="quic_verify mcache depth (config tiles.verify.receive_buffer_size, default.toml:1153)")
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--prelay", action="store_true",
                    help="the producer lays the whole stream into a dcache that holds it before the clock starts "
                         "(tile_run.c TILE_RUN_PRELAY; link depth = the frag count): the stage's rate, not one "
                         "producer core's copy")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES for the tile processes (default: the environment's; at most 32)")
    ap.add_argument("--rocprof", default=None,
                    help="run every tile under rocprofv3 --kernel-trace --stats into this directory")
    ap.add_argument("--walk", action="store_true",
                    help="also time walk mode per tile count: tiles filter every frag (tile_run.c), the link-walk bound")
    ap.add_argument("--timeout", type=float, default=150)
    ap.add_argument("--logdir", default=os.path.join(REPO, "gpurun_out", "tile_bench_logs"))
    args = ap.parse_args()
    if args.build:
        build()
        return
    with tempfile.TemporaryDirectory() as td:
        stream = os.path.join(td, "stream.bin")
        t = time.time()
        s = make_stream(args.frags, stream)
        print(f"stream: {s.n} frags, {s.n_records} signatures, {time.time() - t:.1f} s", file=sys.stderr, flush=True)
        best = None
        if args.walk:
            exe = binary(4096, 2, 0)
            for tiles in (int(x) for x in args.tiles.split(",")):
                depth = 1 << (s.n - 1).bit_length() if args.prelay else args.in_depth
                res = run_one(exe, stream, tiles, depth, args.timeout,
                              os.path.join(args.logdir, f"walk_t{tiles}"), walk=True, prelay=args.prelay)
                print(json.dumps({"walk": True, "tile_cnt": tiles, "frags": s.n, "seconds": res["seconds"],
                                  "frags_walked_per_s": s.n / res["seconds"], "regime": res.get("regime"),
                                  "in_depth": depth, "prelay": args.prelay}), flush=True)
        for cfg in args.configs.split(","):
            exe = binary(*parse_config(cfg))
            b, i, g = parse_config(cfg)
            for tiles in (int(x) for x in args.tiles.split(",")):
                # a GPU-copy tile holds (i + 1) x 2b frags between consuming and the GPU's read, every
                # tiles-th seq: the link must be deeper than that (tile_run.c's producer keeps out of it)
                depth = args.in_depth
                while g and depth < (i + 1) * 2 * b * tiles + 16384:
                    depth *= 2
                if args.prelay:
                    depth = max(depth, 1 << (s.n - 1).bit_length())
                for r in range(args.repeat):
                    res = run_one(exe, stream, tiles, depth, args.timeout,
                                  os.path.join(args.logdir, f"{cfg}_t{tiles}_{r}"), range_mode=is_range(cfg),
                                  prelay=args.prelay, hw_queues=args.hw_queues,
                                  rocprof=os.path.join(args.rocprof, f"{cfg}_t{tiles}_{r}") if args.rocprof else None)
                    res["config"] = cfg
                    res["prelay"] = args.prelay
                    print(json.dumps(res), flush=True)
                    if res.get("overrun"):          # dropped frags: not a valid throughput
                        continue
                    if best is None or res["verifies_per_s"] > best["verifies_per_s"]:
                        best = res
        print(json.dumps({"metric": "ed25519 verifies/sec through the patched reference verify tile (stem_run1, "
                                    "one GPU)", "value": best["verifies_per_s"], "unit": "verifies/s",
                          "config": best["config"], "tiles": best["tile_cnt"], "frags": best["frags"],
                          "sigs": best["sigs"], "in_depth": best["in_depth"], "prelay": args.prelay,
                          "workload": "config 4 stream (firedancer_amd/txn_workload.py), GPU-signed"}))


if __name__ == "__main__":
    main()
