#!/usr/bin/env python3
"""Per-launch timeline of a verify service run, from the GPU tile's rocprofv3
kernel trace (tools/svc_bench.py --rocprof keeps it gzipped for this).

usage: python tools/svc_timeline.py <svc_kernel_trace.csv[.gz]> > timeline.json

A verify launch is the kernels of one launch stream from k_svc_assemble to
k_svc_results.  For each launch: frags (k_svc_assemble's grid), start, end,
the phases (txn kernel, prep, DSM), the DSM's ns per frag, and the share of
the DSM's time a gather (k_svc_gather) or flush (k_svc_compact) ran beside
it.  Run-level: the gaps with no verify kernel, what ran in them, how many
launches overlapped, and the DSM ns per frag against the gather overlap
(split at the median) -- whether sharing the GPU with the PCIe kernels
slows the DSM."""
import csv
import gzip
import json
import statistics
import sys


def base(name):
    return name.split("(")[0].split()[-1].split("<")[0]


def load(path):
    op = gzip.open if path.endswith(".gz") else open
    rows = []
    with op(path, "rt") as f:
        for r in csv.DictReader(f):
            rows.append({"k": base(r["Kernel_Name"]), "s": int(r["Start_Timestamp"]), "e": int(r["End_Timestamp"]),
                         "q": r.get("Stream_Id") or r.get("Queue_Id"), "g": int(r["Grid_Size_X"])})
    rows.sort(key=lambda r: r["s"])
    return rows


def overlap(s, e, iv):
    t = 0
    for a, b in iv:
        if b <= s or a >= e:
            continue
        t += min(b, e) - max(a, s)
    return t


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def main():
    rows = load(sys.argv[1])
    gat = union([(r["s"], r["e"]) for r in rows if r["k"] == "k_svc_gather" and r["g"] > 256])
    fl = union([(r["s"], r["e"]) for r in rows if r["k"] == "k_svc_compact" and r["g"] > 256])
    launches, open_ = [], {}
    for r in rows:
        q = r["q"]
        if r["k"] == "k_svc_assemble":
            open_[q] = {"frags": r["g"], "s": r["s"], "k": {}}
        elif q in open_:
            L = open_[q]
            L["k"].setdefault(r["k"], []).append((r["s"], r["e"]))
            if r["k"] == "k_svc_results":
                L["e"] = r["e"]
                launches.append(L)
                del open_[q]
    launches = [L for L in launches if L["frags"] > 256]         # the warm-up launches are one workgroup
    out = []
    for L in launches:
        d = L["k"].get("k_verify_dsm", [(0, 0)])
        p = L["k"].get("k_verify_prep", [(0, 0)])
        t = L["k"].get("k_txnm_batch", [(0, 0)])
        ds, de = d[0][0], d[-1][1]
        out.append({"frags": L["frags"], "s": L["s"], "e": L["e"], "ms": (L["e"] - L["s"]) / 1e6,
                    "txn_ms": (t[-1][1] - t[0][0]) / 1e6, "prep_ms": (p[-1][1] - p[0][0]) / 1e6,
                    "dsm_ms": (de - ds) / 1e6, "dsm_gather_share": overlap(ds, de, gat) / max(1, de - ds),
                    "dsm_flush_share": overlap(ds, de, fl) / max(1, de - ds)})
    # Grid_Size_X counts threads: k_svc_assemble has one per frag (rounded up to 256)
    for o in out:
        o["dsm_ns_per_frag"] = o["dsm_ms"] * 1e6 / max(1, o["frags"])
    if not out:
        print(json.dumps({"launches": 0}))
        return
    lo, hi = min(o["s"] for o in out), max(o["e"] for o in out)
    ver = union([(o["s"], o["e"]) for o in out])
    gaps = []
    for (a, b), (c, _) in zip(ver, ver[1:]):
        gaps.append((b, c))
    gap_ns = sum(c - b for b, c in gaps)
    conc = sum(1 for i in range(1, len(out)) if out[i]["s"] < max(o["e"] for o in out[:i]))
    med = statistics.median(o["dsm_gather_share"] for o in out)
    lo_g = [o["dsm_ns_per_frag"] for o in out if o["dsm_gather_share"] <= med]
    hi_g = [o["dsm_ns_per_frag"] for o in out if o["dsm_gather_share"] > med]
    summ = {
        "launches": len(out), "span_ms": (hi - lo) / 1e6, "verify_busy_ms": sum(b - a for a, b in ver) / 1e6,
        "gaps": len(gaps), "gap_ms": gap_ns / 1e6,
        "gap_gather_ms": sum(overlap(b, c, gat) for b, c in gaps) / 1e6,
        "gap_flush_ms": sum(overlap(b, c, fl) for b, c in gaps) / 1e6,
        "launches_started_while_another_ran": conc,
        "frags_per_launch_median": statistics.median(o["frags"] for o in out),
        "launch_ms_median": statistics.median(o["ms"] for o in out),
        "prep_ms_median": statistics.median(o["prep_ms"] for o in out),
        "dsm_ms_median": statistics.median(o["dsm_ms"] for o in out),
        "dsm_ns_per_frag_median": statistics.median(o["dsm_ns_per_frag"] for o in out),
        "dsm_gather_share_median": med,
        "dsm_ns_per_frag_low_gather": statistics.median(lo_g) if lo_g else None,
        "dsm_ns_per_frag_high_gather": statistics.median(hi_g) if hi_g else None,
    }
    for o in out:
        o["s"] = (o["s"] - lo) / 1e6
        o["e"] = (o["e"] - lo) / 1e6
    print(json.dumps({"summary": summ, "launches": out}))


if __name__ == "__main__":
    main()
