#!/usr/bin/env python3
"""Run and time the verify stage in service mode (north star's operating
point): the reference's verify tiles patched with
integration/fd_verify_tile_svc.patch (no HIP in the tile processes) served
by one GPU tile (integration/svc_run.c, fd_verify_svc_* in the engine),
between a quic_verify producer and one reliable verify_dedup consumer per
tile (integration/svc_tile_run.c).

Per run: one producer, one GPU-tile process, T tile processes and T
consumer processes, all on one shared file in /dev/shm.

value = signatures the GPU verified for the tiles / (last tile done - first
frag published).  Also: frags/s, outcome counts, per-frag latency (tspub -
tsorig) percentiles, overruns, the service's launch statistics, each
tile's thread count and device fds after privileged_init, and each tile's
published-payload digest (the reference tile's run gives the same digest,
tests/test_gpu_svc_run.py).

usage: python tools/svc_bench.py [--frags N] [--tiles 1,2] [--repeat R] [--rate R,...] [--in-depth D]
       [--gpu-env KEY=VAL,...]
Prints one JSON line per run and a final summary line."""
import argparse
import json
import os
import signal
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))
BUILD = os.path.join(REPO, "integration", "_build")
EXE = os.environ.get("SVC_BENCH_TILE_EXE", os.path.join(BUILD, "svc_tile_run"))   # a build variant for an A/B
SVC = os.path.join(BUILD, "svc_run")


def gpu_numa_node(gpu=0):
    """the NUMA node of the gpu-th AMD GPU (PCI vendor 0x1002, display class), -1 if unknown"""
    try:
        nodes = []
        for d in sorted(os.listdir("/sys/bus/pci/devices")):
            base = os.path.join("/sys/bus/pci/devices", d)
            if open(os.path.join(base, "vendor")).read().strip() == "0x1002" and \
               open(os.path.join(base, "class")).read().strip().startswith(("0x0380", "0x0300", "0x1200")):
                nodes.append(int(open(os.path.join(base, "numa_node")).read().strip()))
        return nodes[gpu] if gpu < len(nodes) else -1
    except (OSError, ValueError):
        return -1


def pick_cpus(count, node=-1):
    """count CPUs of distinct physical cores (one hardware thread each), on
    NUMA node `node` first, among the CPUs this process may use"""
    allowed = sorted(os.sched_getaffinity(0))
    def sib(c):
        try:
            return open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
        except OSError:
            return str(c)
    def on_node(c):
        return node < 0 or os.path.exists(f"/sys/devices/system/cpu/cpu{c}/node{node}")
    seen, first, rest = set(), [], []
    for c in allowed:
        k = sib(c)
        if k in seen:
            continue
        seen.add(k)
        (first if on_node(c) else rest).append(c)
    cpus = (first + rest)[:count]
    return cpus if len(cpus) == count else None


def run_one(stream, tiles, in_depth, timeout, logdir, env=None, svc_env=None, svc_exe=None, gpu=0, pin=None,
            rocprof=None, clients=None):
    """One producer, the GPU tile, `tiles` tile processes and `tiles`
    consumers.  env: the SVC_RUN_* settings (every process); svc_env: the
    GPU tile's (SVC_BATCH_MAX, SVC_INFLIGHT, ...).  Liveness is checked every
    0.2 s: a process that dies ends the run at once.  rocprof: a directory;
    the GPU tile runs under rocprofv3 --kernel-trace --memory-copy-trace
    --stats there (the program itself after --); SVC_BENCH_HIP_TRACE=1 adds
    --hip-trace (the HIP API calls' host durations).  clients: [(name,
    argv)], client processes of the GPU tile beside the verify tiles
    (integration/svc_client.h: a replay or shred harness built with
    FD_HAS_HIP_SVC), client i on the segment's tile tiles + i; each one's
    last stdout line (JSON) lands in res["clients"][name]."""
    shm = f"/dev/shm/fd_svc_bench_{os.getpid()}"
    if os.path.exists(shm):
        os.unlink(shm)
    os.makedirs(logdir, exist_ok=True)
    e = dict(os.environ)
    e.update(env or {})
    clients = list(clients or [])
    if clients:
        e["SVC_RUN_CLIENTS"] = str(len(clients))
    errs, procs = [], []
    # pin: one core each for the producer, the GPU tile, the tiles and the consumers, on the GPU's NUMA node
    # (the reference pins every tile to a core, [layout.affinity]); "auto" picks them, or a list of CPUs
    # the GPU tile gets SVC_CORES cores: the HIP runtime's own threads (the
    # process's signal / callback threads) inherit its affinity, and on one
    # core they take turns with the service loop
    svc_cores = int(os.environ.get("SVC_BENCH_SVC_CORES", "3"))
    if pin == "auto":
        pin = pick_cpus(1 + svc_cores + 2 * tiles, gpu_numa_node(gpu))
    cpu_of = {}
    if pin:
        names = ["producer"] + [f"tile{t}" for t in range(tiles)] + [f"cons{t}" for t in range(tiles)]
        cpu_of = {n: {c} for n, c in zip(names, pin)}
        cpu_of["svc"] = set(pin[1 + 2 * tiles:1 + 2 * tiles + svc_cores])

    def pre(name):
        c = cpu_of.get(name)
        return (lambda: os.sched_setaffinity(0, c)) if c else None

    def spawn(cmd, name, extra=None):
        f = open(os.path.join(logdir, name + ".err"), "w")
        errs.append(f)
        ee = dict(e)
        ee.update(extra or {})
        p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=f, env=ee, preexec_fn=pre(name))
        procs.append((name, p))
        return p

    perr = open(os.path.join(logdir, "producer.err"), "w")
    errs.append(perr)
    prod = subprocess.Popen([EXE, "produce", shm, stream, str(tiles), str(in_depth)], stdout=subprocess.PIPE,
                            stderr=perr, text=True, env=e, preexec_fn=pre("producer"))
    t0 = time.time()
    try:
        line = prod.stdout.readline()
        if line.strip() != "READY":
            raise RuntimeError(f"producer: {line!r} (see {logdir}/producer.err)")
        svc_cmd = [svc_exe or SVC, shm, str(gpu)]
        if rocprof:
            api = ["--hip-trace"] if os.environ.get("SVC_BENCH_HIP_TRACE") else []
            svc_cmd = ["rocprofv3", "--kernel-trace", "--memory-copy-trace"] + api + ["--stats", "--output-format", "csv",
                       "-d", rocprof, "-o", "svc", "--"] + svc_cmd
        spawn(svc_cmd, "svc", svc_env)
        for t in range(tiles):
            spawn([EXE, "consume", shm, str(t)], f"cons{t}")
            spawn([EXE, "tile", shm, str(t)], f"tile{t}")
        cout = {}
        for i, (cname, argv) in enumerate(clients):
            cout[cname] = open(os.path.join(logdir, cname + ".out"), "w+")
            errs.append(cout[cname])
            f = open(os.path.join(logdir, cname + ".err"), "w")
            errs.append(f)
            procs.append((cname, subprocess.Popen(argv, stdout=cout[cname], stderr=f,
                                                  env=dict(e, SVC_CLIENT_SHM=shm, SVC_CLIENT_IDX=str(i)))))
        # a sandboxed tile (SVC_RUN_SANDBOX) dies of SIGSYS after reporting: exit is not in the
        # reference tile's seccomp policy (a reference tile never returns)
        ok_rc = {0, -signal.SIGSYS} if e.get("SVC_RUN_SANDBOX") else {0}

        def bad(n, rc):
            return rc not in (ok_rc if n.startswith("tile") else {0})
        last = 0.0
        while prod.poll() is None:
            dead = [(n, p.returncode) for n, p in procs if p.poll() is not None and bad(n, p.returncode)]
            if dead:
                raise RuntimeError(f"died: {dead} (see {logdir}/*.err)")
            if time.time() - t0 > timeout:
                raise RuntimeError(f"timeout after {timeout} s")
            if time.time() - last >= 10.0:
                print(f"  run: {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
                last = time.time()
            time.sleep(0.2)
        out = prod.stdout.read()
        if prod.returncode:
            raise RuntimeError(f"producer rc {prod.returncode} (see {logdir}/producer.err)")
        for n, p in procs:
            p.wait(timeout=60)
            if bad(n, p.returncode):
                raise RuntimeError(f"{n} rc {p.returncode} (see {logdir}/{n}.err)")
        res = json.loads(out.strip().splitlines()[-1])
        res["pinned"] = {k: sorted(v) for k, v in cpu_of.items()} or None
        if clients:
            res["clients"], res["clients_lines"] = {}, {}
            for cname, f in cout.items():
                f.seek(0)
                lines = [x for x in f.read().splitlines() if x.strip()]
                res["clients"][cname] = json.loads(lines[-1]) if lines else None
                res["clients_lines"][cname] = lines
        return res
    finally:
        # the GPU tile first, with SIGTERM: it stops its IO engine and drains the GPU before it
        # exits (integration/svc_run.c); a process killed with a kernel on the card can leave it faulted
        for n, p in procs:
            if n == "svc" and p.poll() is None:
                p.terminate()
                try:
                    p.wait(timeout=40)
                except subprocess.TimeoutExpired:
                    pass
        for _, p in procs + [("producer", prod)]:
            if p.poll() is None:
                p.kill()
                p.wait()
        for f in errs:
            f.close()
        if os.path.exists(shm):
            os.unlink(shm)


def run_host(clients, logdir, timeout=300, svc_env=None, svc_exe=None, gpu=0, req_depth=128, slot_cap=2048,
             frag_cap=256, env=None):
    """A run of client processes only (svc_tile_run host): the GPU tile (or
    oracle/_ref/svc_mock with svc_exe) and clients [(name, argv)], client i
    on segment tile i.  Returns the host's JSON line with "clients": each
    client's last stdout line (JSON)."""
    shm = f"/dev/shm/fd_svc_host_{os.getpid()}"
    if os.path.exists(shm):
        os.unlink(shm)
    os.makedirs(logdir, exist_ok=True)
    e = dict(os.environ)
    e.update(env or {})
    files, procs = [], []
    herr = open(os.path.join(logdir, "host.err"), "w")
    files.append(herr)
    host = subprocess.Popen([EXE, "host", shm, str(len(clients)), str(req_depth), str(slot_cap), str(frag_cap)],
                            stdout=subprocess.PIPE, stderr=herr, text=True, env=e)
    t0 = time.time()
    try:
        line = host.stdout.readline()
        if line.strip() != "READY":
            raise RuntimeError(f"host: {line!r} (see {logdir}/host.err)")
        f = open(os.path.join(logdir, "svc.err"), "w")
        files.append(f)
        procs.append(("svc", subprocess.Popen([svc_exe or SVC, shm, str(gpu)], stdout=subprocess.DEVNULL, stderr=f,
                                              env=dict(e, **(svc_env or {})))))
        outs = {}
        for i, (cname, argv) in enumerate(clients):
            outs[cname] = open(os.path.join(logdir, cname + ".out"), "w+")
            f = open(os.path.join(logdir, cname + ".err"), "w")
            files += [outs[cname], f]
            procs.append((cname, subprocess.Popen(argv, stdout=outs[cname], stderr=f,
                                                  env=dict(e, SVC_CLIENT_SHM=shm, SVC_CLIENT_IDX=str(i)))))
        while host.poll() is None:
            dead = [(n, p.returncode) for n, p in procs if p.poll() is not None and p.returncode != 0]
            if dead:
                raise RuntimeError(f"died: {dead} (see {logdir}/*.err)")
            if time.time() - t0 > timeout:
                raise RuntimeError(f"timeout after {timeout} s")
            time.sleep(0.1)
        out = host.stdout.read()
        if host.returncode:
            raise RuntimeError(f"host rc {host.returncode} (see {logdir}/host.err)")
        for n, p in procs:
            p.wait(timeout=60)
            if p.returncode:
                raise RuntimeError(f"{n} rc {p.returncode} (see {logdir}/{n}.err)")
        res = json.loads(out.strip().splitlines()[-1])
        res["clients"], res["clients_lines"] = {}, {}
        for cname, f in outs.items():
            f.seek(0)
            lines = [x for x in f.read().splitlines() if x.strip()]
            res["clients"][cname] = json.loads(lines[-1]) if lines else None
            res["clients_lines"][cname] = lines
        return res
    finally:
        for n, p in procs:
            if n == "svc" and p.poll() is None:
                p.terminate()
                try:
                    p.wait(timeout=40)
                except subprocess.TimeoutExpired:
                    pass
        for _, p in procs + [("host", host)]:
            if p.poll() is None:
                p.kill()
                p.wait()
        for f in files:
            f.close()
        if os.path.exists(shm):
            os.unlink(shm)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frags", type=int, default=1 << 21)
    ap.add_argument("--tiles", default="2")
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--in-depth", type=int, default=0,
                    help="quic_verify depth (0: the stream's frag count rounded up, with --prelay)")
    ap.add_argument("--prelay", action="store_true")
    ap.add_argument("--rate", default="0", help="offered rates in frags/s, no flow control (0: flow-controlled)")
    ap.add_argument("--env", default="", help="KEY=VAL,... for every process (SVC_RUN_*)")
    ap.add_argument("--svc-env", default="", help="KEY=VAL,... for the GPU tile (SVC_BATCH_MAX, SVC_INFLIGHT, ...)")
    ap.add_argument("--pin", default="auto", help="auto (one core each on the GPU's NUMA node), none, or c0,c1,...")
    ap.add_argument("--timeout", type=float, default=300)
    ap.add_argument("--rocprof", default=None, help="directory: the GPU tile under rocprofv3 kernel / copy traces")
    ap.add_argument("--logdir", default=os.path.join(REPO, "gpurun_out", "svc_bench_logs"))
    args = ap.parse_args()
    import tile_bench as TB

    def kv(s):
        return dict(x.split("=", 1) for x in s.split(",") if x)
    with tempfile.TemporaryDirectory() as td:
        stream = os.path.join(td, "stream.bin")
        t = time.time()
        s = TB.make_stream(args.frags, stream)
        print(f"stream: {s.n} frags, {s.n_records} signatures, {time.time() - t:.1f} s", file=sys.stderr, flush=True)
        best = None
        for rate in (int(x) for x in args.rate.split(",")):
            for tiles in (int(x) for x in args.tiles.split(",")):
                depth = args.in_depth or (1 << (s.n - 1).bit_length())
                env = kv(args.env)
                if args.prelay:
                    env["SVC_RUN_PRELAY"] = "1"
                    if not args.in_depth:     # prelaid frags with no depth given: a link that holds the stream
                        depth = max(depth, 1 << (s.n - 1).bit_length())
                if rate:
                    env["SVC_RUN_RATE"] = str(rate)
                for r in range(args.repeat):
                    pin = None if args.pin == "none" else args.pin if args.pin == "auto" else [int(x) for x in args.pin.split(",")]
                    res = run_one(stream, tiles, depth, args.timeout, os.path.join(args.logdir, f"t{tiles}_r{rate}_{r}"),
                                  env=env, svc_env=kv(args.svc_env), pin=pin,
                                  rocprof=os.path.join(args.rocprof, f"t{tiles}_{r}") if args.rocprof else None)
                    res["rep"] = r
                    print(json.dumps(res), flush=True)
                    if res.get("overrun") or res.get("lapped"):
                        continue
                    if best is None or res["verifies_per_s"] > best["verifies_per_s"]:
                        best = res
        if best:
            print(json.dumps({"metric": "ed25519 verifies/sec through the service-mode verify stage (one GPU)",
                              "value": best["verifies_per_s"], "tiles": best["tile_cnt"], "frags": best["frags"],
                              "sigs": best["sigs"], "latency": best["latency"]}))


if __name__ == "__main__":
    main()
