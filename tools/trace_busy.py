#!/usr/bin/env python3
"""GPU busy fraction of a C4 run from a rocprofv3 kernel trace.

Usage: python tools/trace_busy.py <run_kernel_trace.csv> <tiles> <warmup> <steps>

The timed region runs from the first k_txn_parse of the timed steps (after
tiles*warmup warmup batches) to the end of the last kernel that starts before
the bench's extra timing batch.  Prints the region's span, the union of kernel
intervals in it (busy), the per-kernel summed durations (kernels on different
streams overlap, so these add up to more than the span) and the HW queues."""
import collections
import csv
import json
import sys


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if ce is not None else 0)


def main():
    path, tiles, warm, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0], r["Queue_Id"])
                for r in csv.DictReader(open(path)))
    parses = [e for e in ev if e[2] == "k_txn_parse"]
    first, after = tiles * warm, tiles * (warm + steps)
    t0 = parses[first][0]
    t1 = max(e[1] for e in ev if e[0] < parses[after][0]) if after < len(parses) else ev[-1][1]
    win = [e for e in ev if e[0] >= t0 and e[1] <= t1]
    per = collections.defaultdict(float)
    for s, e, n, _ in win:
        per[n] += (e - s) / 1e6
    out = {"span_ms": (t1 - t0) / 1e6, "busy_ms": union([(s, e) for s, e, *_ in win]) / 1e6,
           "ms_per_step": (t1 - t0) / 1e6 / steps,
           "kernel_sum_ms": {k: round(v, 3) for k, v in sorted(per.items())},
           "dsm_union_ms": union([(s, e) for s, e, n, _ in win if n == "k_verify_dsm"]) / 1e6,
           "hw_queues": dict(collections.Counter(e[3] for e in win))}
    out["busy_frac"] = out["busy_ms"] / out["span_ms"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
