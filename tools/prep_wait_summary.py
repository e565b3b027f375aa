#!/usr/bin/env python3
"""Summarise tools/run_r03ai.sh (one PMC pass per leg) into per-dispatch means
for k_verify_prep and k_verify_dsm: VALU instructions and issue slots per
wave, issue-slot utilisation, and the share of wave cycles spent waiting
(SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_WAIT_INST_LDS); dispatches under 10% of the
largest one's VALU count (warm-up probes) are left out.
usage: python tools/prep_wait_summary.py gpurun_out/r03ai profiles/r03ai_prep_waits.json"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = ("k_verify_prep", "k_verify_dsm")


def leg(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        return None
    per = collections.defaultdict(lambda: collections.defaultdict(float))   # (kernel, dispatch) -> counter -> value
    for row in csv.DictReader(open(files[0])):
        name = row.get("Kernel_Name", "")
        k = next((k for k in KERNELS if k in name), None)
        if not k:
            continue
        per[(k, row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
    out = {}
    for k in KERNELS:
        ds = [c for (kk, _), c in per.items() if kk == k]
        if not ds:
            continue
        big = max(d["SQ_INSTS_VALU"] for d in ds)       # full batches only (not the warm-up probes)
        ds = [d for d in ds if d["SQ_INSTS_VALU"] >= 0.1 * big]
        m = {c: sum(d[c] for d in ds) / len(ds) for c in ds[0]}
        slots = m["SQ_INSTS_VALU"] - m["SQ_ACTIVE_INST_VALU2"]
        cyc = m["GRBM_GUI_ACTIVE"] / 8.0                      # per XCD
        out[k] = {
            "dispatches": len(ds),
            "valu_insts": m["SQ_INSTS_VALU"],
            "issue_slots": slots,
            "slot_util": round(slots / (1024 * cyc / 4), 4),
            "wait_any_frac": round(m["SQ_WAIT_ANY"] / max(m["SQ_WAVE_CYCLES"], 1.0), 4),
            "wait_inst_any_frac": round(m["SQ_WAIT_INST_ANY"] / max(m["SQ_WAVE_CYCLES"], 1.0), 4),
            "wait_inst_lds_frac": round(m["SQ_WAIT_INST_LDS"] / max(m["SQ_WAVE_CYCLES"], 1.0), 4),
            "lds_insts": m["SQ_INSTS_LDS"],
            "grbm_cycles_per_xcd": cyc,
        }
    return out


def main():
    d, dst = sys.argv[1], sys.argv[2]
    res = {"source": "tools/run_r03ai.sh: rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES "
                     "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE "
                     "GRBM_COUNT --kernel-trace (PMC serialises dispatches); means per dispatch",
           "legs": {}}
    for name in ("c4", "c2"):
        r = leg(os.path.join(d, name))
        if r:
            res["legs"][name] = r
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
