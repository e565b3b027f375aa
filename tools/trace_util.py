#!/usr/bin/env python3
"""Busy time per kernel class from a rocprofv3 kernel trace (run where the
trace is, then keep only this summary: a service run's full trace is
large).

usage: python tools/trace_util.py <dir with *kernel_trace.csv> > util.json

Classes: verify (k_txnm_batch, k_verify_prep, k_verify_dsm, the reduces,
k_msg_order, k_svc_assemble, k_svc_results), ingest (k_svc_gather), flush
(k_svc_compact), other.  For each class: the union of its kernels'
[start, end) intervals (the time at least one ran) and the summed kernel
time; for pairs, the time both ran at once; the span from the first
kernel's start to the last one's end, within the run (first real ingest
to last flush).  The per-kernel ms come from the
trace's own timestamps (ns)."""
import csv
import glob
import json
import os
import sys

CLASSES = {"k_svc_gather": "ingest", "k_svc_compact": "flush"}
VERIFY = ("k_txnm_batch", "k_verify_prep", "k_verify_dsm", "k_seg_reduce", "k_group_reduce", "k_msg_order",
          "k_svc_assemble", "k_svc_results")


def klass(name):
    base = name.split("(")[0].split()[-1].split("<")[0]
    if base in CLASSES:
        return CLASSES[base]
    return "verify" if base in VERIFY else "other"


def union(iv):
    iv = sorted(iv)
    out, cs, ce = [], None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                out.append((cs, ce))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        out.append((cs, ce))
    return out


def length(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append((s, e))
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def main():
    files = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), klass(r["Kernel_Name"]), int(r["Grid_Size_X"])))
    # the run: from the first real ingest (the warm-up launches are one workgroup) to the last flush
    ing = [s for s, e, c, g in rows if c == "ingest" and g > 256]
    fl = [e for s, e, c, g in rows if c == "flush"]
    lo, hi = (min(ing), max(fl)) if ing and fl else (0, 1 << 62)
    iv, tot = {}, {}
    for s, e, c, g in rows:
        s, e = max(s, lo), min(e, hi)
        if s >= e:
            continue
        iv.setdefault(c, []).append((s, e))
        tot[c] = tot.get(c, 0) + (e - s)
    allk = [x for v in iv.values() for x in v]
    span = (max(e for _, e in allk) - min(s for s, _ in allk)) if allk else 0
    u = {c: union(v) for c, v in iv.items()}
    out = {"span_ms": span / 1e6, "classes": {}}
    for c in u:
        out["classes"][c] = {"busy_ms": length(u[c]) / 1e6, "kernel_ms": tot[c] / 1e6, "kernels": len(iv[c])}
    names = sorted(u)
    out["both_ms"] = {f"{a}+{b}": length(intersect(u[a], u[b])) / 1e6 for i, a in enumerate(names) for b in names[i + 1:]}
    out["any_ms"] = length(union(allk)) / 1e6
    print(json.dumps(out))


if __name__ == "__main__":
    main()
