#!/usr/bin/env python3
"""Summarise tools/run_valu_calib.sh (one rocprofv3 PMC pass over the VALU
microbenchmark tools/valu_rates2 and over bench.py --contexts 1) into
profiles/<tag>_valu_issue_calibration.json.

What it establishes (gfx950, hardware counters, no clock assumption):
  * SQ_INSTS_VALU counts wave-instructions; SQ_ACTIVE_INST_VALU2 counts the
    quad-cycles in which a SIMD issued TWO VALU instructions (dual issue).
    Issue slots used = INSTS_VALU - ACTIVE_INST_VALU2 (one slot = one
    quad-cycle of one SIMD with at least one VALU issue).
  * capacity = SIMDs (1024) x GRBM_GUI_ACTIVE/8 (cycles per XCD) / 4.
  * slot utilisation = used / capacity <= 1 by construction.
  * per instruction class: wave-instructions per cycle per SIMD (ipc) and
    the dual-issue share -- which classes can pair (v_add_u32, v_and/or/xor,
    v_lshrrev_b32, v_mov, f32 add/fma) and which cannot (VOP3 integer ops,
    carry chains, v_mad_u64_u32, v_lshlrev_b32, v_cndmask).
usage: python tools/valu_calib_summary.py gpurun_out/valu_<tag> profiles/<tag>_valu_issue_calibration.json
"""
import collections
import csv
import json
import os
import sys

SIMDS = 1024


def load(d):
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        x = disp[r["Dispatch_Id"]]
        x[r["Counter_Name"]] = float(r["Counter_Value"])
        x["kernel"] = r["Kernel_Name"].split("(")[0]
        x["grid"] = int(r.get("Grid_Size", 0) or 0)
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        if r["Dispatch_Id"] in disp:
            disp[r["Dispatch_Id"]]["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    return disp


def derive(x):
    n, v2, g = x["SQ_INSTS_VALU"], x["SQ_ACTIVE_INST_VALU2"], x["GRBM_GUI_ACTIVE"]
    cyc = g / 8.0
    out = {"valu_insts": n, "dual_issue_quads": v2, "issue_slots": n - v2,
           "grbm_cycles_per_xcd": cyc, "ipc_per_simd": n / (cyc * SIMDS),
           "dual_issue_share": v2 / n if n else 0.0, "slot_util": (n - v2) / (SIMDS * cyc / 4.0),
           "int32_share": x["SQ_INSTS_VALU_INT32"] / n if n else 0.0,
           "int64_share": x["SQ_INSTS_VALU_INT64"] / n if n else 0.0}
    if "ms" in x:
        out["ms"] = x["ms"]
        out["held_clock_ghz"] = cyc / (x["ms"] * 1e-3) / 1e9
    return out


def main():
    d, out = sys.argv[1], sys.argv[2]
    res = {"source": f"{d}: rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU "
                     "SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_BUSY_CYCLES SQ_WAVES "
                     "GRBM_GUI_ACTIVE GRBM_COUNT (one pass) --kernel-trace",
           "definition": "issue slots = SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2; slot_util = slots / "
                         "(1024 SIMDs x GRBM_GUI_ACTIVE/8 / 4)",
           "microbench_8_waves_per_simd": {}, "engine": {}}
    micro = load(os.path.join(d, "micro"))
    best = {}
    for x in micro.values():
        k = x["kernel"]
        if k.startswith("k_") and (k not in best or x["grid"] > best[k]["grid"]):
            best[k] = x
    for k, x in sorted(best.items()):
        res["microbench_8_waves_per_simd"][k[2:]] = {kk: round(v, 4) for kk, v in derive(x).items()
                                                    if kk in ("ipc_per_simd", "dual_issue_share", "slot_util",
                                                              "int32_share", "int64_share")}
    eng = load(os.path.join(d, "engine"))
    for k in ("k_verify_prep", "k_verify_dsm"):
        xs = [derive(x) for x in eng.values() if x["kernel"] == k]
        if xs:
            res["engine"][k] = {kk: round(sum(x[kk] for x in xs) / len(xs), 4 if kk != "valu_insts" else 0)
                                for kk in xs[0]}
            res["engine"][k]["dispatches"] = len(xs)
    single = [v["slot_util"] for v in res["microbench_8_waves_per_simd"].values() if v["dual_issue_share"] < 0.01
              and v["ipc_per_simd"] > 0.1]
    res["single_issue_ceiling_slot_util"] = round(max(single), 4) if single else None
    # which machine code these counters describe (bench.py checks it against the loaded library)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from firedancer_amd.kernel_hash import kernel_hashes
    res["kernel_sha"] = kernel_hashes(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                   "firedancer_amd", "libfd_ed25519_hip.so"))
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["engine"], indent=1))
    print("single-issue microbench ceiling:", res["single_issue_ceiling_slot_util"])


if __name__ == "__main__":
    main()
