#!/usr/bin/env python3
"""bench.py -- ed25519 verifies/s on MI355X (BASELINE.json metric), one JSON line.

A step is one verify pass (k_verify_prep + k_verify_dsm) over one batch of
2^20 signatures resident in HBM, split over two verify contexts (HIP
streams) so that one half's prep fills the issue slots the other half's DSM
leaves idle at its end (--contexts; the verdicts are checked against a
whole-batch pass through one context): BASELINE config 2 ("same 1M-sig batch on one
MI355X with 10% corrupted sigs plus non-canonical R/A, S>=L and small-order
points"), 64-byte messages, keys/signatures generated on the GPU by the
engine's own signer, mutated with the C2 model (firedancer_amd/workload.py).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
one process per GPU, each verifies its own 2^20-signature shard (weak scaling,
no data-path collective: signatures are independent); RCCL is used only for
the barrier and the max-over-ranks time.

Roofline: VALU issue (the kernels are integer-VALU bound).
gfx950 issues at most one VALU wave-instruction per SIMD per quad-cycle,
plus a second one in the same quad-cycle only for "dual-issue" e32 ops from
another wave (v_add_u32, v_and/or/xor, v_mov, ...; never v_mad_u64_u32, VOP3
integer ops or carry chains -- profiles/r02a_valu_issue_calibration.json).
So the roofline of k_verify_dsm is its issue slots, counted by hardware:
slots = SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2 per launch (rocprofv3 PMC pass of
this build), against 1024 SIMDs x clock / 4.  "frac" = achieved / peak at
the clock the chip holds under this load (GRBM_GUI_ACTIVE per XCD / kernel
time, same pass): <= 1 by construction; frac_at_max_clock prices the same
slots against the 2.4 GHz maximum.  The single-issue microbenchmark reaches
~0.95 of the slots (launch ramp included).  See issue_roofline().

SURVEY 8(d)'s W (the reference algorithm's int32-op count, 7.33e5 per verify
at 64 B; W_dsm = 6.08e5 for the part k_verify_dsm does) is kept as
ref_work_rate_vs_peak = units x W_dsm / time / 78.6 Tops/s: a speed-up over
the reference algorithm (the half-size kernel executes ~17% less), not a
utilisation.  The kernel duration is measured live with HIP events on the
launch stream.

cpu_baseline (rank 0, every N, after the timed region): the reference's own fd_ed25519_verify (AVX-512
IFMA build, compiled from the reference sources into oracle/_ref/) on a
bounded 65536-record sample of the same batch, one pinned thread per core.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "ed25519 verifies/sec (1/2/4/8 MI355X) + % of INT32 VALU peak"
N_M, N_S = 1378.6, 1518.1
N_M_DECODE, N_S_DECODE = 42.0, 510.0
PEAK_OPS = 256 * 4 * 32 * 2.4e9          # 78.6e12 int32 lane-ops/s (32-wide SIMDs)
SIMDS, MAX_CLOCK = 256 * 4, 2.4e9         # MI355X_MICROARCH.md: 256 CU x 4 SIMD, 2400 MHz max clock
PEAK_SLOTS = SIMDS * MAX_CLOCK / 4        # VALU issue slots/s: one quad-cycle per SIMD at the max clock
PMC_SUMMARY = "r06af_pmc_summary.json"   # rocprofv3 PMC passes of this kernel build (tools/run_profile.sh)
ISSUE_SUMMARY = "r06af_valu_issue_calibration.json"   # VALU issue-slot pass of this build (tools/run_valu_calib.sh)
ISSUE_SUMMARY_C4 = "r06af_c4_valu_issue.json"         # the same pass over C4's timing-leg batch (tools/run_c4_issue.sh)
PMC_SUMMARY_C4 = "r06af_c4_pmc_summary.json"           # FETCH/WRITE passes over the C4 bench (tools/txnm_pmc_summary.py)


def w_total(msg_sz):
    nblk = -(-(msg_sz + 81) // 128)
    return 304 * N_M + 200 * N_S + 4900 * nblk


W_DSM = 304 * (N_M - N_M_DECODE) + 200 * (N_S - N_S_DECODE)


def c5_shard(sigs_per_rank, rank, world):
    """Config 5: 2^26 signatures in total (or sigs_per_rank * world), cut
    into contiguous shard_bounds ranges, one per rank.
    Returns (total, lo, hi)."""
    from firedancer_amd.shard import shard_bounds
    total = sigs_per_rank * world if sigs_per_rank else 1 << 26
    lo, hi = shard_bounds(total, rank, world)
    return total, lo, hi


ISSUE_UNITS = 933793      # survivors per launch in that pass (the C2 2^20 batch, seed 0x5eed0001: deterministic)


def profile_build_check(summary):
    """Does the committed profile summary describe the kernels of the library
    this run loaded?  Compares the gfx950 machine-code hashes the summary
    records (firedancer_amd/kernel_hash.py) with the loaded library's."""
    want = summary.get("kernel_sha") or {}
    try:
        from firedancer_amd.kernel_hash import engine_kernel_hashes
        have = engine_kernel_hashes()
    except Exception as e:                     # noqa: BLE001 -- reported, never fatal to the bench line
        return {"profile_matches_build": None, "kernel_sha_error": str(e)}
    keys = [k for k in ("k_verify_dsm", "k_verify_prep") if k in want]
    ok = bool(keys) and all(want[k] == have.get(k) for k in keys)
    return {"profile_matches_build": ok, "kernel_sha": {k: have.get(k) for k in keys},
            "profile_kernel_sha": {k: want[k] for k in keys}}


def issue_roofline(dsm_avg_ms, units_per_launch, summary=ISSUE_SUMMARY):
    """VALU issue roofline of k_verify_dsm from the committed PMC pass of this
    build (profiles/ISSUE_SUMMARY, tools/run_valu_calib.sh):
      slots per launch  = SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2 (quad-cycles of a
                          SIMD with >= 1 VALU issue; dual-issued pairs count once)
      cycles per launch = GRBM_GUI_ACTIVE / 8 (per XCD), same pass
      achieved          = slots per launch / live launch time (HIP events)
      held clock        = cycles per launch / live launch time (the kernel is
                          issue-bound: its cycle count, not its time, is what
                          stays fixed from run to run as the clock moves)
      peak              = 1024 SIMDs x held clock / 4 (one issue slot per
                          quad-cycle per SIMD)
      frac              = achieved / peak = slots / (1024 x cycles / 4): the
                          counters' own ratio (pmc_frac), <= 1 by construction
      frac_at_max_clock = achieved / (1024 x 2.4 GHz / 4)
    DESIGN.md 6 states the formula; the single-issue microbenchmark ceiling
    (tools/valu_rates2 under the same counters) is ~0.95."""
    path = os.path.join(REPO, "profiles", summary)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        cal = json.load(f)
    e = cal["engine"]["k_verify_dsm"]
    units_ref = e.get("units", ISSUE_UNITS)
    scale = units_per_launch / units_ref             # exact (1) for the profiled batch; per-survivor scaling otherwise
    slots, cycles = e["issue_slots"] * scale, e["grbm_cycles_per_xcd"] * scale
    t = dsm_avg_ms * 1e-3
    achieved = slots / t
    clock = cycles / t                               # the launch's cycle count over its live duration
    peak = SIMDS * clock / 4
    return {"bound": "valu_issue", "unit": "T issue-slots/s", "achieved": round(achieved / 1e12, 5),
            "peak": round(peak / 1e12, 5), "frac": round(achieved / peak, 4), "pmc_frac": e["slot_util"],
            "frac_at_max_clock": round(achieved / PEAK_SLOTS, 4), "held_clock_ghz": round(clock / 1e9, 4),
            "held_clock_ghz_pmc_pass": e["held_clock_ghz"],
            "issue_slots_per_launch": round(slots), "dual_issue_share": e["dual_issue_share"],
            "slots_scaled_from_c2": summary == ISSUE_SUMMARY and abs(units_per_launch - units_ref) > 0.5,
            "slots_scaled_from_profiled_units": abs(units_per_launch - units_ref) > 0.5,
            **profile_build_check(cal),
            "single_issue_ceiling": cal.get("single_issue_ceiling_slot_util"),
            "issue_source": f"profiles/{summary} (rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 "
                            "GRBM_GUI_ACTIVE ..., one pass, " +
                            ("bench.py --config c4, the timing leg's dispatch)" if summary == ISSUE_SUMMARY_C4
                             else "bench.py --contexts 1)")}


def c4_issue_roofline(dsm_avg_ms, units_per_launch):
    """C4 reads its own PMC pass when one of this build is committed (the
    unit counts agree: the C4 stream is deterministic); otherwise C2's,
    scaled per survivor (slots_scaled_from_c2 true)."""
    path = os.path.join(REPO, "profiles", ISSUE_SUMMARY_C4)
    if os.path.exists(path):
        r = issue_roofline(dsm_avg_ms, units_per_launch, ISSUE_SUMMARY_C4)
        if r and r.get("profile_matches_build") and not r["slots_scaled_from_profiled_units"]:
            return r
    return issue_roofline(dsm_avg_ms, units_per_launch)


def ingest_roofline(st):
    """HBM roofline of the verify tile's frag-ingest kernel (k_txnm_batch:
    during_frag's copy, after_frag's parse, record expansion) for tile 0's
    timing-leg batch: algorithmic bytes (fd_verify_hip_tile_ingest_stats,
    include/fd_verify_hip.h) / kernel time (HIP events) against 8 TB/s; the
    traffic is the committed PMC pass's FETCH_SIZE x 2 + WRITE_SIZE per
    launch (profiles/PMC_SUMMARY_C4) when it describes this build's kernel."""
    if not st or not st["ms"]:
        return None
    achieved = st["bytes"] / (st["ms"] * 1e-3) / 1e9
    r = {"kernel": "k_txnm_batch<16>", "bound": "hbm", "unit": "GB/s", "achieved": round(achieved, 1),
         "peak": 8000.0, "frac": round(achieved / 8000.0, 4), "avg_launch_ms": round(st["ms"], 4),
         "algorithmic_bytes_per_launch": st["bytes"], "frags_per_launch": st["frags"], "records": st["records"],
         "traffic": None}
    path = os.path.join(REPO, "profiles", PMC_SUMMARY_C4)
    if os.path.exists(path):
        with open(path) as f:
            pm = json.load(f)
        k = pm.get("kernels", {}).get("k_txnm_batch")
        have = None
        try:
            from firedancer_amd.kernel_hash import engine_kernel_hashes
            have = engine_kernel_hashes(names=("k_txnm_batch<16>",)).get("k_txnm_batch<16>")
        except Exception:                          # noqa: BLE001 -- reported as no match
            pass
        if k:
            # the PMC pass profiles whole 2^20-frag launches (one tile); this
            # leg's launch is one tile's share of a step, so the traffic is
            # that pass's bytes per algorithmic byte times this launch's
            ratio = k["hbm_side_bytes_per_launch"] / k["algorithmic_bytes_per_launch"]
            r["traffic"] = round(ratio * st["bytes"], 1)
            r["traffic_ratio"] = round(ratio, 3)
            r["traffic_source"] = (f"profiles/{PMC_SUMMARY_C4}: FETCH_SIZE*2 + WRITE_SIZE of k_txnm_batch over "
                                   f"{k.get('frags_per_launch')}-frag launches ({k['hbm_side_bytes_per_launch']:.0f} B "
                                   f"per launch), scaled to this launch by bytes per algorithmic byte")
            r["profile_matches_build"] = bool(have) and have == pm.get("kernel_sha", {}).get("k_txnm_batch<16>")
    return r


def prep_issue_util():
    """k_verify_prep's issue-slot utilisation from the same PMC pass (counters only)."""
    path = os.path.join(REPO, "profiles", ISSUE_SUMMARY)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)["engine"]["k_verify_prep"]["slot_util"]


def write_fdv1(path, sigs, pubs, pool, moff, msz):
    with open(path, "wb") as f:
        f.write(b"FDV1")
        f.write(np.array([sigs.shape[0], pool.size, 0], np.uint64).tobytes())
        f.write(np.ascontiguousarray(sigs).tobytes()); f.write(np.ascontiguousarray(pubs).tobytes())
        f.write(np.ascontiguousarray(moff, np.uint32).tobytes()); f.write(np.ascontiguousarray(msz, np.uint32).tobytes())
        f.write(np.ascontiguousarray(pool).tobytes())


def cpu_baseline(sigs, pubs, pool, moff, msz, gpu_codes, threads, target_s):
    """Time the reference's own verify on the host (bounded sample)."""
    has_ifma = "avx512ifma" in open("/proc/cpuinfo").read()
    exe = os.path.join(REPO, "oracle", "_ref", "ref_cpu_bench_avx512" if has_ifma else "ref_cpu_bench_ref")
    kind, backend = "reference", ("avx512" if has_ifma else "portable")
    if not os.path.exists(exe):
        return {"value": None, "unit": "verifies/s", "cores": 0, "kind": "reference",
                "sample": "unavailable: oracle/_ref not built on this box"}
    with tempfile.TemporaryDirectory() as td:
        inp = os.path.join(td, "in.bin"); out = os.path.join(td, "codes.bin")
        write_fdv1(inp, sigs, pubs, pool, moff, msz)
        # one core, short pass: per-core rate and calibration
        r1 = json.loads(subprocess.check_output([exe, inp, "1", "-", "0", "1"], timeout=600).decode())
        rate1 = r1["rate"]
        n = sigs.shape[0]
        rep = max(1, int(round(target_s * rate1 * threads / n)))
        r = json.loads(subprocess.check_output([exe, inp, str(threads), out, "0", str(rep)], timeout=900).decode())
        ref_codes = np.fromfile(out, np.int8)
    return {"value": round(r["rate"], 1), "unit": "verifies/s", "cores": threads, "kind": kind,
            "backend": backend, "per_core": round(rate1, 1),
            "sample": f"{n} records of the same C2 batch x {rep} passes ({r['verifies']} verifies, "
                      f"{r['seconds']:.2f} s wall, {threads} pinned threads)",
            "bitmap_match": bool(np.array_equal(ref_codes == 0, gpu_codes == 0)),
            "codes_match": bool(np.array_equal(ref_codes, gpu_codes))}


_JSON_FD = [1]
COLL_DEV = None          # device of the tensors the collectives reduce (GPU for RCCL, CPU for gloo)


def emit(out):
    """The one JSON line, on the real stdout (see _quiet_stdout)."""
    os.write(_JSON_FD[0], (json.dumps(out) + "\n").encode())


def _quiet_stdout():
    """RCCL prints its version banner to stdout when a communicator is created;
    route fd 1 to stderr for the run and keep the real stdout for emit()."""
    sys.stdout.flush()
    _JSON_FD[0] = os.dup(1)
    os.dup2(2, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5"],
                    help="BASELINE.json configs: c1 all-valid 2^20/GPU; c2 (default, the metric's config) "
                         "C2 mix 2^20/GPU; c3 one 32-B message x 2^22 keys/GPU as batch_single_msg "
                         "groups of 16; c4 synthetic txn stream through the verify tile (GPU parse + verify + "
                         "host tcache dedup); c5 2^26 C2-mix signatures in total, sharded (strong scaling)")
    ap.add_argument("--txns", type=int, default=1 << 20,
                    help="c4: frags per step per GPU (2^20: 102-106M verifies/s; 2^19 under-fills the DSM launches, "
                         "84-99M -- profiles/r02c_c4_sweep)")
    ap.add_argument("--halfsize", type=int, default=1, choices=[0, 1],
                    help="0: full-length scalars (k, 1) in k_verify_dsm, an A/B switch (same verdicts)")
    ap.add_argument("--contexts", type=int, default=2,
                    help="c1/c2/c3/c5: verify contexts (streams) each step is split over (measured with the "
                         "persistent DSM: 1 -> 118.2M, 2 -> 125.0-125.7M, 4 -> 124.5M verifies/s)")
    ap.add_argument("--tiles", type=int, default=6,
                    help="c4: verify tiles (host threads + contexts) per GPU (r02n, 2^20 frags per step, resident / "
                         "PCIe-inclusive M verifies/s: 2 -> 101-103 / 75-85, 4 -> 100-102 / 90-95, 6 -> 106-109 / "
                         "98-101, 8 -> 100-102 / 97-98)")
    ap.add_argument("--dsm-share", type=int, default=1,
                    help="c4: each tile's k_verify_dsm grid is 1/share of the resident slots, so that many "
                         "tiles' DSM launches share the GPU")
    ap.add_argument("--c4-ingest", default="frags", choices=["frags", "payload"],
                    help="c4: fd_txn_m_t frags in each tile's in-link dcache (default) or raw payloads + offsets")
    ap.add_argument("--c4-pcie", default="dma", choices=["zerocopy", "dma", "dma_tile_stream"],
                    help="c4 PCIe-inclusive leg: the GPU reads each in-link dcache in place from pinned mapped host "
                         "memory (zerocopy), or it is copied host->HBM each step on a copy stream per tile (dma) or "
                         "on the tile's own stream ahead of its batch (dma_tile_stream)")
    ap.add_argument("--c4-pcie-steps", type=int, default=24,
                    help="c4 PCIe-inclusive leg: timed steps (the pipeline's fill, one copy, and drain, one host "
                         "pass, are paid once per leg; 0: --steps)")
    ap.add_argument("--sigs", type=int, default=None, help="override signatures per GPU per step")
    ap.add_argument("--no-c4", action="store_true",
                    help="c2 (default config): skip the config-4 sub-object (the verify-tile path, 'c4' in the line)")
    ap.add_argument("--no-tile", action="store_true",
                    help="skip the patched reference verify tile leg (out['tile'], rank 0 at N=1)")
    ap.add_argument("--tile-frags", type=int, default=1 << 22)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dump-codes", default=None, help="c1/c2/c3/c5: each rank saves its codes to <prefix>.<rank>.npy")
    ap.add_argument("--force-dist", action="store_true", help="init torch.distributed even at world size 1")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (RCCL over xGMI, one rank per GPU: the driver's N-GPU runs); gloo rehearses the "
                         "N>1 path with several ranks sharing one GPU (rank r on GPU r %% device_count)")
    args = ap.parse_args()
    if args.config == "c4" or (args.config == "c2" and not args.no_c4):
        # The reference runs each verify tile as its own process, each with the
        # HIP runtime's own hardware queues; here the tiles are threads of one
        # process, so give that process a queue per tile (HIP default 4).
        # Resident C4 is unchanged, the PCIe-inclusive leg +6% (profiles/r03u:
        # 113.8/113.6 vs 113.8/114.5 M resident, 100.6/100.9 vs 106.4/106.5 M).
        # Set before the runtime initialises (the torch import below).  The
        # GPU boxes export HIP's default of 4 (profiles/r05af/host.txt), and
        # it is left in place: this process keeps its queues while the tile
        # leg's GPU tile runs beside it, and 8 here plus 16 there made the
        # paced tile runs lose most frags (profiles/r05ah; alone, r05ai: none).
        os.environ.setdefault("GPU_MAX_HW_QUEUES", str(max(4, min(args.tiles + 2, 8))))

    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    global COLL_DEV
    if world > 1 or args.force_dist:
        import torch.distributed as dist
        _quiet_stdout()
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            COLL_DEV = torch.device("cuda", local)
        else:
            dist.init_process_group("gloo")
            COLL_DEV = torch.device("cpu")

    from firedancer_amd import Verifier
    from firedancer_amd.ed25519 import CTX_STREAM
    from firedancer_amd.workload import make_batch_gpu, make_batch_gpu_range

    cfg = args.config
    if cfg == "c4":
        return run_c4(args, rank, world, local, dist)
    msg_sz = 32 if cfg == "c3" else 64
    mix = "c1" if cfg in ("c1", "c3") else "c2"
    scaling = "weak"
    if cfg == "c5":
        total, lo, hi = c5_shard(args.sigs, rank, world)
        n = hi - lo
        scaling = "strong"
    else:
        n = args.sigs or ((1 << 22) if cfg == "c3" else (1 << 20))
    chunk = min(n, 1 << 20)
    v = Verifier(device=local, chunk_sigs=chunk)      # signs the batch; runs the roofline leg
    if cfg == "c5":
        # this rank's shard of one global seeded set: a one-process pass over
        # [0, total) verifies the same records (workload.range_inputs)
        batch = make_batch_gpu_range(v, lo, hi, msg_sz=msg_sz, mix=mix)
    else:
        batch = make_batch_gpu(v, n, msg_sz=msg_sz, seed=0x5eed0001 + 7919 * rank, mix=mix,
                               shared_msg=(cfg == "c3"))
    dev = batch.dev
    codes = torch.zeros(n, dtype=torch.int8, device=dev)
    bitmap = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    gcodes = torch.zeros((n + 15) // 16, dtype=torch.int8, device=dev)

    # Each step's batch is split over C verify contexts (one HIP stream each),
    # as the reference spreads a stream of transactions over several verify
    # tiles: with no synchronisation between steps, one context's prep runs in
    # the issue slots another's k_verify_dsm leaves idle in its last partial
    # round of workgroups.  Slices are multiples of 256 signatures (whole
    # bitmap words and whole 16-signature groups).
    C = max(1, args.contexts)
    per = ((n + C - 1) // C + 255) // 256 * 256
    slices = [(lo, min(n, lo + per)) for lo in range(0, n, per)]
    ctxs = [Verifier(device=local, chunk_sigs=min(hi - lo, 1 << 20)) for lo, hi in slices]
    for vv in ctxs + [v]:
        vv.set_halfsize(args.halfsize)

    def groups_of(lo, hi):   # fd_ed25519_verify_batch_single_msg in chunks of 16 (fd_ed25519_user.c:238-241)
        ng = (hi - lo + 15) // 16
        first = torch.arange(ng, dtype=torch.int32, device=dev) * 16
        cnt = torch.clamp((hi - lo) - first, max=16).to(torch.uint8)
        return ng, first, cnt, gcodes[lo // 16:lo // 16 + ng]

    jobs = [(vv, lo, hi, groups_of(lo, hi) if cfg == "c3" else None) for vv, (lo, hi) in zip(ctxs, slices)]
    whole = [(v, 0, n, groups_of(0, n) if cfg == "c3" else None)]

    def step(jl):
        # each context on its own stream (CTX_STREAM), so the contexts overlap;
        # the inputs were made on torch's stream and synchronised before warmup
        for vv, lo, hi, g in jl:
            vv.verify_dev(hi - lo, batch.sigs[lo:hi], batch.pubs[lo:hi], batch.pool, batch.msg_off[lo:hi],
                          batch.msg_sz[lo:hi], codes[lo:hi], bitmap[lo // 64:(hi + 63) // 64], stream=CTX_STREAM)
            if g:
                vv.group_reduce_dev(g[0], g[1], g[2], codes[lo:hi], g[3], stream=CTX_STREAM)

    def sync_all():
        for vv in ctxs + [v]:
            vv.sync()
        torch.cuda.synchronize()

    torch.cuda.synchronize()          # batch generation (torch stream) before the context streams read it
    for _ in range(args.warmup):
        step(jobs)
    sync_all()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(jobs)
    sync_all()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    timed_codes, timed_gcodes = codes.clone(), gcodes.clone()
    # roofline leg: the whole batch through one context with HIP events around
    # every launch (timing mode), so each k_verify_dsm runs alone on the GPU;
    # its verdicts must equal the timed multi-context steps'
    v.set_timing(True)
    for _ in range(max(1, min(args.steps, 3))):
        step(whole)
    sync_all()
    prep_ms, dsm_ms, launches = v.get_timing()
    v.set_timing(False)
    assert torch.equal(codes, timed_codes) and torch.equal(gcodes, timed_gcodes), "contexts != whole batch"
    elapsed = t1 - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=COLL_DEV)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    c = codes.cpu().numpy()
    if args.dump_codes:                       # this rank's verdicts, for the shard-vs-whole-set checks
        np.save(f"{args.dump_codes}.{rank}.npy", c)
    bm = bitmap.cpu().numpy().view(np.uint64)
    bits = np.unpackbits(bm.view(np.uint8), bitorder="little")[:n].astype(bool)
    assert np.array_equal(bits, c == 0), "bitmap != codes"
    reached_dsm = int(np.isin(c, (0, -3)).sum())          # passed every pre-check
    accept = float((c == 0).mean())

    if dist:
        nt = torch.tensor([n], dtype=torch.int64, device=COLL_DEV)
        dist.all_reduce(nt)
        n_all = int(nt.item())
    else:
        n_all = n
    total = n_all * args.steps
    value = total / elapsed
    launches_per_step = -(-n // chunk)
    dsm_avg_ms = dsm_ms / max(launches, 1)
    prep_avg_ms = prep_ms / max(launches, 1)
    units_per_launch = reached_dsm / launches_per_step
    # T int32-ops/s per GPU: SURVEY 8(d)'s per-unit W (the reference
    # algorithm's work), and the kernel's own smaller half-size work
    achieved = units_per_launch * W_DSM / (dsm_avg_ms * 1e-3) / 1e12
    peak = PEAK_OPS / 1e12
    # whole pipeline (prep + DSM): the prep work (decodes + hash) for every
    # signature, the DSM work only for those that pass the pre-checks
    pipe_s = (prep_avg_ms + dsm_avg_ms) * 1e-3 * max(launches_per_step, 1)
    w_prep = w_total(msg_sz) - W_DSM
    pipeline_frac = (n * w_prep + reached_dsm * W_DSM) / pipe_s / PEAK_OPS

    # HBM-side bytes per k_verify_dsm launch from the committed rocprofv3 PMC
    # passes of this same command (FETCH_SIZE x2 per the gfx950 note + WRITE_SIZE)
    issue = issue_roofline(dsm_avg_ms, units_per_launch)
    traffic, traffic_src = None, None
    pmc = os.path.join(REPO, "profiles", PMC_SUMMARY)
    if cfg == "c2" and n == (1 << 20) and os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f)["kernels"]["k_verify_dsm"]["derived"]["hbm_side_bytes_per_launch"]
        traffic_src = f"profiles/{PMC_SUMMARY}: FETCH_SIZE*2 + WRITE_SIZE of k_verify_dsm (rocprofv3 --pmc)"
    ingest_bytes = 64 + 32 + msg_sz + 8                   # sig, pub, msg, off/sz per signature
    ingest_gbps = n / launches_per_step * ingest_bytes / (prep_avg_ms * 1e-3) / 1e9

    out = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline:          # rank 0, after every rank's timed region
            k = min(65536, n)
            idx = slice(0, k)
            sigs = batch.sigs[idx].cpu().numpy(); pubs = batch.pubs[idx].cpu().numpy()
            moff = batch.msg_off[idx].cpu().numpy().view(np.uint32)
            msz = batch.msg_sz[idx].cpu().numpy().view(np.uint32)
            lo = int(moff.min()); hi = int((moff.astype(np.int64) + msz).max())
            pool = batch.pool[lo:hi].cpu().numpy()
            threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
            cpu = cpu_baseline(sigs, pubs, pool, moff - lo, msz, c[idx], threads, args.cpu_seconds)
            cpu["sample"] = cpu.get("sample", "") + f" [{cfg}]"
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "verifies/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (GPU-signed random keys, C2 mutation model)",
            "config": {"workload": {
                           "c1": f"config 1: {n} sigs/GPU, 64-B msgs, all valid",
                           "c2": f"config 2: {n} sigs/GPU, 64-B msgs, C2 validity mix",
                           "c3": f"config 3: one 32-B msg x {n} keys/GPU, batch_single_msg groups of 16",
                           "c5": f"config 5: {n_all} C2-mix sigs total, {n} on rank 0"}[cfg],
                       "config_id": cfg, "sigs_per_gpu": n, "msg_sz": msg_sz,
                       "parallelism": f"dp{world} (signature shards)",
                       "verify_contexts": len(ctxs)},
            "accept_rate": round(accept, 5),
            "roofline": dict(issue or {}, **{
                         "kernel": "k_verify_dsm", "traffic": traffic, "traffic_unit": "bytes/launch",
                         "traffic_source": traffic_src, "units_per_launch": round(units_per_launch),
                         "avg_launch_ms": round(dsm_avg_ms, 4),
                         "ref_work_rate_vs_peak": round(achieved / peak, 4),
                         "ref_work_note": "SURVEY 8(d)'s W (the reference algorithm's full-length-scalar work, "
                                          f"{round(W_DSM)} int32-op equivalents per unit) x units / time / 78.6 "
                                          "Tops/s: a speed-up figure over the reference algorithm, NOT a "
                                          "utilisation (the half-size kernel does 17% less work, so it can pass 1)",
                         "timing_leg": "after the timed steps: the whole batch through one context, HIP events "
                                       "around each launch, each k_verify_dsm alone on the GPU"}),
            "pipeline": {"prep_ms": round(prep_avg_ms, 4), "dsm_ms": round(dsm_avg_ms, 4),
                         "prep_issue_slot_util": prep_issue_util(),
                         "w_total_per_verify": round(w_total(msg_sz)),
                         "ref_work_rate_vs_peak": round(pipeline_frac, 4),
                         "ref_work_note": "prep work (decodes + hash) for every signature, DSM work for those "
                                          "reaching it, at 8(d)'s W, over the prep + DSM time: a speed-up figure "
                                          "over the reference algorithm, not a utilisation",
                         "ingest_GBps": round(ingest_gbps, 2), "ingest_bytes_per_sig": ingest_bytes},
            "cpu_baseline": cpu,
        }
    for vv in ctxs + [v]:
        vv.close()
    if cfg == "c2" and not args.no_c4:
        # config 4, the north star's workload (the verify tile's frags), as a
        # sub-object of the same line: every rank runs it after the C2 leg
        c4 = run_c4(args, rank, world, local, dist, emit_line=False)
        if rank == 0:
            out["c4"] = {k: c4[k] for k in ("value", "unit", "ms_per_step", "steps", "frags_per_s", "config",
                                            "frag_outcomes_last_batch", "batch_gpu_ms", "batch_host_ms",
                                            "roofline", "ingest_roofline", "pcie_inclusive", "cpu_baseline")}
    if cfg == "c2" and not args.no_tile and rank == 0 and world == 1:
        out["tile"] = run_tile_leg(args)
        cb = (out.get("c4") or {}).get("cpu_baseline")
        if cb and cb.get("value"):               # the same C4 workload through the reference's own CPU tile
            out["tile"]["cpu_baseline"] = dict(cb, note="the c4 leg's: the reference's verify tile on host cores, "
                                                        "over the same C4 stream shape")
    if rank == 0:
        emit(out)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return out


def run_tile_leg(args):
    """The north star's operating point in service mode: the reference's
    verify tiles with integration/fd_verify_tile_svc.patch (single-threaded,
    no HIP, the reference's sandbox possible) in the reference's stem_run1
    loop, served by one GPU tile per GPU (integration/svc_run.c:
    fd_verify_svc_*, every tile's requests merged into one launch), between a
    quic_verify producer and a reliable verify_dedup consumer per tile
    (integration/svc_tile_run.c, tools/svc_bench.py), over --tile-frags frags
    of the C4 stream.

    value: the highest drop-free rate on the reference's link: a paced
    producer with no flow control (quic_verify is unreliable,
    src/app/fdctl/topology.c:173) on an mcache of the reference's default
    depth (16384, default.toml:1153), the rate bisected between the
    flow-controlled rate of the same shape and 2 M frags/s
    (tools/svc_link_sweep.py: drop_free_search), each probed rate judged
    by the majority of up to 3 runs (judge_rate: one run's collapse does not
    decide a step; every run is listed in tried); value = the signatures per
    second of a drop-free run at the highest passing rate, with its tspub - tsorig p50/p99 and the frags
    lost at 1.2x.  The frags are prelaid in the dcache (one producer core's
    copy caps near 15-20 M frags/s); the mcache still laps a slow tile.  Both
    request forms are searched: range (the tile posts mcache ranges, the GPU
    tile's engine reads the link) and polled (during_frag copies each frag
    into the segment's frag area, as the reference's during_frag copies it
    into the tile's scratch, fd_verify_tile.c:64-99).  parity: a run whose
    consumers digest every published frag, each tile's digest and counts
    against the reference's own parse and AVX-512 verify over that tile's
    share (oracle/_ref/libfdref_txn.so ref_verify_tile_digest).  prelaid: the
    round-5 headline, kept as a secondary field: flow-controlled on a link
    deep enough to hold the stream.  Binaries are built from the reference
    sources in the build container (integration/_build); without them the
    leg reports why and the line goes on."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    sys.path.insert(0, os.path.join(REPO, "tests"))
    try:
        import tempfile
        import svc_bench as SB
        import svc_io as SI
        import svc_link_sweep as SL
        import tile_bench as TB
        if not (os.path.exists(SB.EXE) and os.path.exists(SB.SVC)):
            return {"value": None, "error": "integration/_build/svc_tile_run or svc_run missing (build() with /root/reference)"}
        # the reference's default verify_tile_count (default.toml:776); FD_BENCH_TILE_TILES=3 is round 6's
        # earlier shape (profiles/r06/final)
        tiles = int(os.environ.get("FD_BENCH_TILE_TILES", "6"))
        DEPTH = 16384
        # request slots for a shallow link: many small ranges
        paced_env = {"SVC_RUN_PRELAY": "1", "SVC_RUN_REQ_DEPTH": os.environ.get("FD_BENCH_TILE_REQ_DEPTH", "128"),
                     "SVC_RUN_SLOT_CAP": os.environ.get("FD_BENCH_TILE_SLOT_CAP", "2048")}
        with tempfile.TemporaryDirectory() as td:
            stream = os.path.join(td, "stream.bin")
            s = TB.make_stream(args.tile_frags, stream)
            # FD_BENCH_TILE_LOGDIR: keep every run's process logs (a GPU box's gpurun_out/...)
            logdir = os.environ.get("FD_BENCH_TILE_LOGDIR") or os.path.join(td, "logs")
            nrun = [0]

            def run(depth, env, rate=0):
                nrun[0] += 1
                e = dict(env, SVC_RUN_RATE=str(int(rate))) if rate else dict(env)
                rd = os.path.join(logdir, f"run{nrun[0]}")
                try:
                    return SB.run_one(stream, tiles, depth, 180, rd, env=e, pin="auto",
                                      svc_env={"SVC_DEBUG_S": "10"})
                except Exception as x:          # name the run and what its processes said last
                    tails = {}
                    for f in sorted(os.listdir(rd)) if os.path.isdir(rd) else []:
                        with open(os.path.join(rd, f), errors="replace") as fh:
                            t = fh.read()[-600:]
                        if t.strip():
                            tails[f] = t
                    raise RuntimeError(f"run {nrun[0]} (depth {depth}, rate {int(rate)}, "
                                       f"{ {k: v for k, v in env.items() if k != 'SVC_RUN_PRELAY'} }): {x}; logs: {tails}")

            def lat(r):
                return {"offered_frags_per_s": int(r["offered_rate"]), "achieved_verifies_per_s": r["verifies_per_s"],
                        "frags_per_s": r["frags_per_s"], "lost": SL.lost(r),
                        "p50_us": r["latency"]["p50_us"], "p99_us": r["latency"]["p99_us"],
                        "p999_us": r["latency"]["p999_us"]}

            forms = {}
            for form, extra in (("range", {}), ("polled", {"SVC_RUN_POLLED": "1"})):
                env = dict(paced_env, **extra)
                fc = run(DEPTH, env)                       # flow-controlled: the shape's own rate
                best, tried = SL.drop_free_search(lambda rate: run(DEPTH, env, rate), fc["frags_per_s"], 2e6, 4,
                                                  votes=3)
                over = run(DEPTH, env, 1.2 * best["offered_rate"]) if best else None
                forms[form] = {"flow_controlled_frags_per_s": fc["frags_per_s"],
                               "drop_free": lat(best) if best else None,
                               "at_1p2": lat(over) if over else None,
                               "tried": [lat(r) for _, r in tried]}
            head = max((f for f in forms if forms[f]["drop_free"]),
                       key=lambda f: forms[f]["drop_free"]["achieved_verifies_per_s"], default=None)
            hd = forms[head]["drop_free"] if head else None
            # parity against the reference's code, per tile (flow-controlled, every frag digested)
            depth_all = 1 << (s.n - 1).bit_length()
            # deep-link shape: 32768-frag slots, as many as the service's 4 GiB staging holds (16 at 3 tiles,
            # 8 at 6: fd_verify_svc_boot_ok, 2176 B of staging per frag)
            req_deep = 16
            while tiles * req_deep * 32768 * 2176 >= 1 << 32:
                req_deep //= 2
            pre = {"SVC_RUN_PRELAY": "1", "SVC_RUN_REQ_DEPTH": str(req_deep), "SVC_RUN_SLOT_CAP": "32768"}
            d = run(depth_all, dict(pre, SVC_RUN_DIGEST="1"))
            ref = SI.ref_share_digests(s.pool, s.off, s.sz, None, tiles, 0x7f4a11, 4194302, threads=16)
            got = [SI.tile_counts(x) for x in d["tiles"]]
            equal = all(g == {k: r[k] for k in g} for g, r in zip(got, ref)) and d["consumer_bad"] == 0
            # secondary: round 5's prelaid number, flow-controlled on a link that holds the stream
            wins = [run(depth_all, pre) for _ in range(3)]
            wmed = sorted(wins, key=lambda x: x["verifies_per_s"])[1]
        return {"value": hd["achieved_verifies_per_s"] if hd and equal else None, "unit": "verifies/s",
                "frags_per_s": hd["frags_per_s"] if hd else None,
                "offered_frags_per_s": hd["offered_frags_per_s"] if hd else None,
                "latency_us": {"p50": hd["p50_us"], "p99": hd["p99_us"], "p999": hd["p999_us"]} if hd else None,
                "form": head, "forms": forms,
                "parity": {"frags_compared": d["frags"], "tiles": tiles, "equal": bool(equal),
                           "against": "the reference's fd_txn_parse + AVX-512 fd_ed25519_verify_batch_single_msg "
                                      "over each tile's share, tcache and bundle pass in arrival order"},
                "prelaid": {"value": wmed["verifies_per_s"], "frags_per_s": wmed["frags_per_s"], "in_depth": depth_all,
                            "windows": [round(x["verifies_per_s"], 1) for x in wins],
                            "overrun": sum(x["overrun"] + x["lapped"] for x in wins),
                            "req_depth": req_deep, "slot_cap": 32768,
                            "what": "flow-controlled, a link that holds the whole stream (round 5's headline)"},
                "svc": wmed["svc"], "regime": wmed["regime"],
                "tile_process": {"threads_max": wmed["tile_threads_max"], "dev_fds": wmed["tile_dev_fds"]},
                "config": {"tiles": tiles, "gpus": 1, "in_depth": DEPTH, "paced_env": paced_env,
                           "workload": f"config 4 stream, {s.n} frags ({s.n_records} signatures), GPU-signed"},
                "what": "fd_verify_tile.c + integration/fd_verify_tile_svc.patch in stem_run1 (svc_tile_run.c), "
                        "unreliable paced producer at quic_verify depth 16384 -> tile processes (no HIP) -> consumers, "
                        "one GPU tile process (svc_run.c); value = the signatures/s of the highest drop-free rate"}
    except Exception as e:                   # the tile leg never fails the bench line
        return {"value": None, "error": f"{type(e).__name__}: {e}"}


def ref_tile_baseline(pool, off, sz, threads, target_s, seed, depth):
    """The reference's verify tile path (fd_txn_parse + fd_txn_verify with its
    tcache, compiled from the reference sources) on T pinned host threads, one
    tile per thread, frags round-robined by seq like before_frag."""
    import ctypes
    path = os.path.join(REPO, "oracle", "_ref", "libfdref_txn.so")
    if not os.path.exists(path):
        return {"value": None, "unit": "verifies/s", "cores": 0, "kind": "reference",
                "sample": "unavailable: oracle/_ref not built on this box"}
    L = ctypes.CDLL(path)
    c = ctypes
    L.ref_verify_tile_bench.argtypes = [c.c_int, c.c_int, c.c_uint64, c.c_uint64, c.c_uint64, c.c_uint64,
                                        c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p]
    n = off.size
    res = np.zeros(n, np.int8)
    o = np.zeros(4, np.float64)
    L.ref_verify_tile_bench(1, 0, 1, seed, depth, n, pool.ctypes.data, off.ctypes.data, sz.ctypes.data,
                            res.ctypes.data, o.ctypes.data)
    per_core = o[2] / o[0]
    rep = max(1, int(round(target_s * per_core * threads / max(o[2], 1))))
    L.ref_verify_tile_bench(threads, 0, rep, seed, depth, n, pool.ctypes.data, off.ctypes.data, sz.ctypes.data,
                            res.ctypes.data, o.ctypes.data)
    return {"value": round(o[2] / o[0], 1), "unit": "verifies/s", "cores": threads, "kind": "reference",
            "per_core": round(per_core, 1), "frags_per_s": round(o[1] / o[0], 1),
            "sample": f"first {n} frags of the same stream x {rep} passes ({int(o[2])} signatures, {o[0]:.2f} s wall, "
                      f"{threads} pinned threads = {threads} verify tiles, tcache depth {depth} each)"}


def run_c4(args, rank, world, local, dist, emit_line=True):
    """Config 4: synthetic Solana txn stream through the verify tile.

    A step is one batch of --txns frags through --tiles GPU verify tiles
    (fd_verify_hip_tile) sharing the GPU, the frags split round robin between
    them as the reference splits them between its verify tiles
    (fd_verify_tile.c before_frag: seq % round_robin_cnt).  Ingest (--c4-ingest):
      frags    (default) the tile's own format: each tile's in-link dcache of
               fd_txn_m_t frags (src/disco/fd_txn_m.h) in HBM; the GPU does
               during_frag's copy into the out dcache and after_frag's parse
               in place (fd_verify_hip_tile_submit_frags)
      payload  raw payloads + caller-marshalled offsets (round 1's path)
    Each tile owns a context (stream), a tcache of depth 4194302 (the
    reference default signature_cache_size) and a host thread, and runs GPU
    ingest/parse + sig0 tag + record expansion + verify + per-txn
    batch_single_msg reduce, then the ordered host pass (tcache dedup,
    bundle state).  Batches are submitted one ahead, so a tile's host pass of
    batch k overlaps the GPU work of batch k+1.  Each step re-keys the dedup
    hash so the replayed batch is new traffic to the tcache (once a tcache is
    full every insert also evicts, the steady state of a long-running tile);
    in-batch resends still dedup.
    value = signatures verified per second (all tiles, all ranks), in-link
    dcaches resident in HBM.  A second timed leg (frags ingest) copies every
    tile's in-link dcache host->HBM each step from pinned memory on a copy
    stream, triple-buffered and queued one batch ahead, so the copy of batch
    k+1 overlaps the GPU work of batch k and the host pass of batch k-1:
    "pcie_inclusive"."""
    import threading

    import torch
    from firedancer_amd import Verifier
    from firedancer_amd.ed25519 import CTX_STREAM, HostBuffer
    from firedancer_amd.txn_workload import PARSED_CHUNKS, gpu_signer, make_txn_stream, txnm_dcache
    from firedancer_amd.verify_tile import IN_QUIC, VerifyTile
    T = max(1, args.tiles)
    frags_mode = args.c4_ingest == "frags"
    v = Verifier(device=local, chunk_sigs=1 << 20)
    seed_base = 0x7f4a11 + 104729 * rank
    s = make_txn_stream(args.txns, gpu_signer(v), seed=0x5eed0004 + 7919 * rank)
    dev = torch.device("cuda", local)
    depth = 4194302
    vs = [v] + [Verifier(device=local, chunk_sigs=1 << 16) for _ in range(T - 1)]
    for vv in vs:
        vv.set_dsm_share(args.dsm_share)
    to_dev = lambda a, view=None: torch.from_numpy(np.ascontiguousarray(a if view is None else a.view(view))).to(dev)
    parts, h2d_bytes = [], 0
    d_pool = None if frags_mode else to_dev(s.pool)
    for t in range(T):
        sel = np.arange(t, s.n, T)
        if frags_mode:
            region, chunk, fsz = txnm_dcache(s.pool, s.off[sel], s.sz[sel], seed=t + 1)
            hb = HostBuffer(region.size)                     # pinned, device-mapped (fd_ed25519_hip_host_alloc)
            hb.array[:] = region
            h_in = torch.from_numpy(hb.array)
            d_in = [to_dev(region), torch.empty_like(h_in, device=dev), torch.empty_like(h_in, device=dev)]
            d_out = torch.empty(64 * PARSED_CHUNKS * max(int(sel.size), 1), dtype=torch.uint8, device=dev)
            out_chunk = to_dev((np.arange(sel.size) * PARSED_CHUNKS).astype(np.uint32), np.int32)
            kinds = to_dev(np.full(sel.size, IN_QUIC, np.uint8))
            parts.append(dict(n=int(sel.size), hb=hb, h_in=h_in, d_in=d_in, d_out=d_out,
                              in_chunk=to_dev(chunk, np.int32),
                              in_sz=to_dev(fsz, np.int16), kinds=kinds, out_chunk=out_chunk,
                              cs=torch.cuda.Stream(dev), ts=torch.cuda.ExternalStream(vs[t].stream, device=dev),
                              free=[None] * 3, ready=[None] * 3))
            h2d_bytes += region.size
        else:
            parts.append(dict(n=int(sel.size), off=to_dev(s.off[sel], np.int32), sz=to_dev(s.sz[sel], np.int16)))
    tiles = [VerifyTile(vs[t], max_txn=parts[t]["n"], hashmap_seed=seed_base, tcache_depth=depth) for t in range(T)]
    k_step = [0] * T
    diag = os.environ.get("FD_C4_DIAG")
    h2d = [False]

    def stage(t, j):
        # copy step j's in-link dcache host -> HBM on the tile's copy stream
        # (pinned, DMA engine) into buffer j % 3, once batch j-3's GPU work
        # (the buffer's previous reader) is done
        P = parts[t]
        b = j % 3
        with torch.cuda.stream(P["cs"]):
            if P["free"][b] is not None:
                P["cs"].wait_event(P["free"][b])
            P["d_in"][b].copy_(P["h_in"], non_blocking=True)
            ready = torch.cuda.Event()
            ready.record(P["cs"])
        P["ready"][b] = (j, ready)

    def submit(t, more=False):
        P = parts[t]
        tiles[t].set_seed(seed_base + 7 * k_step[t])
        if not frags_mode:
            tiles[t].submit(P["n"], d_pool, P["off"], P["sz"])
        elif not h2d[0]:
            tiles[t].submit_frags(P["n"], P["d_in"][0], P["in_chunk"], P["in_sz"], P["kinds"], P["d_out"],
                                  P["out_chunk"])
        elif args.c4_pcie == "zerocopy":
            # the ingest kernel reads the in-link dcache in place over PCIe
            tiles[t].submit_frags(P["n"], P["hb"].ptr, P["in_chunk"], P["in_sz"], P["kinds"], P["d_out"],
                                  P["out_chunk"])
        elif args.c4_pcie == "dma_tile_stream":
            # the copy is queued on the tile's own stream right before its batch:
            # no extra stream (hardware queues are shared beyond 4 per process);
            # the other tile's GPU work overlaps it
            buf = P["d_in"][k_step[t] & 1]
            vs[t].stage_async(buf, P["hb"], P["hb"].nbytes, stream=CTX_STREAM)
            tiles[t].submit_frags(P["n"], buf, P["in_chunk"], P["in_sz"], P["kinds"], P["d_out"], P["out_chunk"])
        else:
            # the batch waits for its staged copy; the next batch's copy is
            # queued right behind this submit, so it overlaps this batch's GPU
            # work and the host pass of the one before (triple-buffered)
            j = k_step[t]
            b = j % 3
            if P["ready"][b] is None or P["ready"][b][0] != j:
                stage(t, j)
            P["ts"].wait_event(P["ready"][b][1])
            tiles[t].submit_frags(P["n"], P["d_in"][b], P["in_chunk"], P["in_sz"], P["kinds"], P["d_out"],
                                  P["out_chunk"])
            done = torch.cuda.Event()
            done.record(P["ts"])
            P["free"][b] = done
            if more:
                stage(t, j + 1)
        k_step[t] += 1

    def tile_loop(t, steps, outs, gpu_ms, host_ms):
        submit(t, more=steps > 1)
        for k in range(steps):
            if k + 1 < steps:
                submit(t, more=k + 2 < steps)
            outs[t].append(tiles[t].complete())
            lt = tiles[t].last_timing(); gpu_ms[t].append(lt["gpu_ms"]); host_ms[t].append(lt["host_ms"])
            if diag:
                print(f"c4 tile {t} step {k}: gpu batch {lt['gpu_ms']:.3f} ms, host pass {lt['host_ms']:.3f} ms",
                      file=sys.stderr)

    def run(steps):
        outs, gpu_ms, host_ms = [[] for _ in range(T)], [[] for _ in range(T)], [[] for _ in range(T)]
        th = [threading.Thread(target=tile_loop, args=(t, steps, outs, gpu_ms, host_ms)) for t in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        return outs, gpu_ms, host_ms

    def metrics():
        ms = [tl.metrics() for tl in tiles]
        return {k: sum(m[k] for m in ms) for k in ms[0]}

    def timed(steps):
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        m0 = metrics()
        t0 = time.perf_counter()
        outs, gpu_ms, host_ms = run(steps)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        m1 = metrics()
        sigs = m1["sigs"] - m0["sigs"]
        frags = s.n * steps
        if dist:
            t = torch.tensor([elapsed], dtype=torch.float64, device=COLL_DEV)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            tt = torch.tensor([sigs, frags], dtype=torch.int64, device=COLL_DEV)
            dist.all_reduce(tt)
            sigs, frags = int(tt[0].item()), int(tt[1].item())
        return elapsed, sigs, frags, outs, gpu_ms, host_ms, m1["sigs"] - m0["sigs"]

    torch.cuda.synchronize()          # uploads before the tile streams read them
    run(max(args.warmup, 1))
    elapsed, sigs, frags, outs, gpu_ms, host_ms, my_sigs = timed(args.steps)
    pcie = None
    if frags_mode:
        h2d[0] = True
        run(1)
        k2 = args.c4_pcie_steps or args.steps
        e2, sigs2, _, outs2, _, _, _ = timed(k2)
        same = all(np.array_equal(a[-1][0], b[-1][0]) for a, b in zip(outs, outs2))
        pcie = {"value": round(sigs2 / e2, 1), "unit": "verifies/s", "steps": k2, "ms_per_step": round(e2 / k2 * 1e3, 4),
                "h2d_bytes_per_step": h2d_bytes * world, "h2d_GBps": round(h2d_bytes * world * k2 / e2 / 1e9, 2),
                "results_equal_resident_leg": bool(same),
                "mode": args.c4_pcie,
                "what": ("every tile's in-link dcache (fd_txn_m_t frags) in pinned device-mapped host memory, read in "
                         "place by the ingest kernel over PCIe each step" if args.c4_pcie == "zerocopy" else
                         "every tile's in-link dcache (fd_txn_m_t frags) copied host->HBM each step from pinned memory "
                         + ("on the tile's own stream ahead of its batch" if args.c4_pcie == "dma_tile_stream" else
                            "(copy stream per tile, triple-buffered, queued one batch ahead)")) +
                        "; per-frag results D2H as in the resident leg; the out dcache stays in HBM"}
        h2d[0] = False
    res = np.concatenate([o[-1][0] for o in outs])
    gpu_ms = [x for g in gpu_ms for x in g]; host_ms = [x for h in host_ms for x in h]
    # kernel roofline: one extra (untimed) batch of tile 0 with per-kernel HIP-event timing
    v.set_timing(True)
    tiles[0].set_ingest_timing(frags_mode)
    submit(0); tiles[0].complete()
    prep_ms, dsm_ms, launches = v.get_timing()
    dsm_units = v.get_dsm_units()
    ing = tiles[0].ingest_stats() if frags_mode else None
    tiles[0].set_ingest_timing(False)
    v.set_timing(False)
    n_sig_batch = int(my_sigs) // max(args.steps, 1)
    launches = max(launches, 1)
    out = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline:          # rank 0, after every rank's timed region
            k = min(32768, s.n)
            hi = int((s.off[:k].astype(np.int64) + s.sz[:k]).max())
            threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
            cpu = ref_tile_baseline(s.pool[:hi + 64].copy(), s.off[:k].copy(), s.sz[:k].copy(), threads,
                                    args.cpu_seconds, seed_base, depth)
        counts = {int(a): int(b) for a, b in zip(*np.unique(res, return_counts=True))}
        names = {0: "publish", -1: "verify_fail", -2: "dedup", -3: "parse_fail", -4: "bundle_peer_fail"}
        dsm_avg = dsm_ms / launches
        achieved = dsm_units / launches * W_DSM / (dsm_avg * 1e-3) / 1e12
        out = {
            "metric": METRIC,
            "value": round(sigs / elapsed, 1),
            "unit": "verifies/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic txn stream (repo generator, GPU-signed, C2 mutation per signature, "
                    "1% resends, 0.1% grafted sig0, 0.5% malformed)",
            "config": {"workload": f"config 4: {s.n} frags/GPU/batch ({n_sig_batch} signatures), legacy+v0 txns "
                                   f"1-12 sigs, <=1232 B, GPU fd_txn_parse, {T} verify tiles (round robin), "
                                   f"tcache dedup depth {depth} each",
                       "config_id": "c4", "frags_per_gpu": s.n, "sigs_per_batch": n_sig_batch, "verify_tiles": T,
                       "parallelism": f"dp{world} (frag shards; {T} verify tiles per GPU)", "dsm_share": args.dsm_share},
            "frags_per_s": round(frags / elapsed, 1),
            "frag_outcomes_last_batch": {names[k]: v_ for k, v_ in counts.items()},
            "batch_gpu_ms": round(float(np.median(gpu_ms)), 4),
            "batch_host_ms": round(float(np.median(host_ms)), 4),
            "roofline": dict(c4_issue_roofline(dsm_avg, dsm_units / launches) or {}, **{
                         "kernel": "k_verify_dsm", "traffic": None, "units_per_launch": round(dsm_units / launches),
                         "ref_work_rate_vs_peak": round(achieved / (PEAK_OPS / 1e12), 4),
                         "avg_launch_ms": round(dsm_avg, 4), "launches_per_batch": launches,
                         "prep_ms_per_batch": round(prep_ms, 4),
                         "timing_leg": "one extra batch of tile 0 alone, HIP events around each launch"}),
            "ingest": args.c4_ingest,
            "ingest_roofline": ingest_roofline(ing),
            "pcie_inclusive": pcie,
            "cpu_baseline": cpu,
        }
        if emit_line:
            emit(out)
    for tl in tiles:
        tl.close()
    for x in vs:
        x.close()
    for P in parts:
        if "hb" in P:
            P["h_in"] = None
            P["hb"].close()
    if dist and emit_line:
        dist.barrier()
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
