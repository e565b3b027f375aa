#!/usr/bin/env python3
"""The service-mode verify stage under the reference's link conditions: an
unreliable quic_verify producer (no flow control, topology.c:173) paced at
an offered rate, at several link depths (tiles.verify.receive_buffer_size;
the reference's default is 16384).

Per depth:
- the highest drop-free rate: bisection over the offered rate between
  --lo and the flow-controlled rate of the same run shape (a rate is
  drop-free when no frag is overrun or lapped);
- the overruns at 1.2x that rate (the fraction of frags lost);
- the per-frag latency (mcache tsorig to the tile's publish, and to the
  consumer's read) at the drop-free rate, p50 / p99.

The frags are prelaid in the dcache (SVC_RUN_PRELAY: one producer core's
copy would otherwise cap the offered rate); the mcache keeps `depth`
lines, so a producer that laps a tile overruns it as on the reference's
link.  Each run is integration/svc_tile_run.c through tools/svc_bench.py's
run_one (pinned: one core each on the GPU's NUMA node).

usage: python tools/svc_link_sweep.py [--frags N] [--tiles T] [--depths 16384,65536,262144] [--steps S]
Prints one JSON line per run, then one line per depth and a markdown table
on stderr."""
import argparse
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import svc_bench as SB  # noqa: E402


def lost(r):
    """frags the stage lost: overrun or lapped on a range link, or never seen by a tile (a polled
    link's overruns are counted by the stem, not the tile: integration/svc_tile_run.c "unseen")"""
    return r["overrun"] + r["lapped"] + r.get("unseen", 0)


def judge_rate(run, rate, tried, votes=3):
    """Whether rate is drop-free: the majority of up to `votes` runs at it
    lose no frag (runs stop once the majority is decided: 2 agreeing runs of
    3).  A single run's collapse (r06y: one 7.6 M frags/s run lost 190 K of
    4.19 M frags between drop-free runs at 29 M's neighbours) then no longer
    decides a bisection step alone.  Every run goes into tried.  Returns
    (passed, a drop-free run at this rate or None)."""
    ok, bad, good = 0, 0, None
    need = votes // 2 + 1
    while ok < need and bad < need:
        r = run(rate)
        tried.append((rate, r))
        if lost(r):
            bad += 1
        else:
            ok += 1
            good = good or r
    return ok >= need, good


def drop_free_search(run, hi, lo, steps, votes=1):
    """The highest offered rate in [lo, hi] at which run(rate) loses no frag:
    hi first, then a geometric bisection (the rates span a decade).  With
    votes > 1 each rate is judged by the majority of up to `votes` runs
    (judge_rate).  Returns (best run or None, every run as (rate, run))."""
    tried = []
    passed, r = judge_rate(run, hi, tried, votes)
    if passed:
        return r, tried
    best = None
    for _ in range(steps):
        mid = (lo * hi) ** 0.5
        passed, r = judge_rate(run, mid, tried, votes)
        if passed:
            lo, best = mid, r
        else:
            hi = mid
    if best is None:
        passed, r = judge_rate(run, lo, tried, votes)
        best = r if passed else None
    return best, tried


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frags", type=int, default=1 << 22)
    ap.add_argument("--tiles", type=int, default=2)
    ap.add_argument("--depths", default="16384,65536,262144")
    ap.add_argument("--steps", type=int, default=5, help="bisection steps per depth")
    ap.add_argument("--lo", type=float, default=2e6, help="lowest offered rate, frags/s")
    ap.add_argument("--env", default="", help="KEY=VAL,... for every process (SVC_RUN_*)")
    ap.add_argument("--svc-env", default="", help="KEY=VAL,... for the GPU tile only")
    ap.add_argument("--pin", default="auto")
    ap.add_argument("--timeout", type=float, default=120)
    ap.add_argument("--votes", type=int, default=3, help="runs per probed rate, majority decides (judge_rate)")
    ap.add_argument("--mock", action="store_true", help="the CPU stand-in for the GPU tile (oracle/_ref/svc_mock)")
    ap.add_argument("--logdir", default=os.path.join(SB.REPO, "gpurun_out", "svc_link_sweep_logs"))
    args = ap.parse_args()
    import tile_bench as TB
    base_env = dict(x.split("=", 1) for x in args.env.split(",") if x)
    base_env["SVC_RUN_PRELAY"] = "1"
    svc_env = dict(x.split("=", 1) for x in args.svc_env.split(",") if x)
    pin = None if args.pin == "none" else "auto"
    runs = [0]

    def run(stream, depth, rate):
        env = dict(base_env)
        if rate:
            env["SVC_RUN_RATE"] = str(int(rate))
        runs[0] += 1
        r = SB.run_one(stream, args.tiles, depth, args.timeout, os.path.join(args.logdir, f"run{runs[0]}"),
                       env=env, svc_env=svc_env, pin=pin, svc_exe=os.path.join(SB.REPO, "oracle", "_ref", "svc_mock") if args.mock else None)
        line = {k: r[k] for k in ("in_depth", "offered_rate", "frags", "overrun", "lapped", "verifies_per_s",
                                  "frags_per_s", "latency", "latency_to_consumer")}
        line["stream_frags"] = r["stream_frags"]
        print(json.dumps(line), flush=True)
        return r

    rows = []
    with tempfile.TemporaryDirectory() as td:
        stream = os.path.join(td, "stream.bin")
        t = time.time()
        if args.mock:                                         # no GPU: the oracle signs a small stream
            import numpy as np
            import txn_lib as T
            from firedancer_amd.txn_workload import make_txn_stream
            from tile_io import write_fdt1
            s = make_txn_stream(args.frags, T.oracle_signer, seed=0x7e6b)
            write_fdt1(stream, s.pool, s.off, s.sz, np.zeros(s.n, np.uint64), 0x5eed7117, 1 << 14)
        else:
            s = TB.make_stream(args.frags, stream)
        print(f"stream: {s.n} frags, {time.time() - t:.1f} s", file=sys.stderr, flush=True)
        for depth in (int(x) for x in args.depths.split(",")):
            fc = run(stream, depth, 0)                       # flow-controlled: the stage's own rate
            best, _ = drop_free_search(lambda rate: run(stream, depth, rate), fc["frags_per_s"], args.lo, args.steps,
                                       votes=args.votes)
            if best is None:
                best = run(stream, depth, args.lo)
            over = run(stream, depth, 1.2 * best["offered_rate"])
            row = {"depth": depth, "tiles": args.tiles, "flow_controlled_frags_per_s": fc["frags_per_s"],
                   "drop_free_rate": best["offered_rate"], "drop_free_lost": lost(best),
                   "drop_free_verifies_per_s": best["verifies_per_s"],
                   "p50_us": best["latency"]["p50_us"], "p99_us": best["latency"]["p99_us"],
                   "p50_to_consumer_us": best["latency_to_consumer"]["p50_us"],
                   "p99_to_consumer_us": best["latency_to_consumer"]["p99_us"],
                   "rate_1p2": over["offered_rate"], "lost_1p2": lost(over),
                   "lost_frac_1p2": lost(over) / max(1, over["stream_frags"])}
            rows.append(row)
            print(json.dumps({"depth_summary": row}), flush=True)
    print("| depth | flow-controlled (M frags/s) | highest drop-free rate (M frags/s) | latency p50 / p99 (us) "
          "| to consumer p50 / p99 (us) | lost at 1.2x |", file=sys.stderr)
    print("|---|---|---|---|---|---|", file=sys.stderr)
    for w in rows:
        print(f"| {w['depth']} | {w['flow_controlled_frags_per_s'] / 1e6:.1f} | {w['drop_free_rate'] / 1e6:.1f} "
              f"| {w['p50_us']:.0f} / {w['p99_us']:.0f} | {w['p50_to_consumer_us']:.0f} / {w['p99_to_consumer_us']:.0f} "
              f"| {w['lost_1p2']} ({100 * w['lost_frac_1p2']:.1f} %) |", file=sys.stderr)


if __name__ == "__main__":
    main()
