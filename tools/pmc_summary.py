#!/usr/bin/env python3
"""Summarise tools/run_profile.sh output (rocprofv3 kernel stats + PMC passes)
into one JSON per round: per-kernel mean counter values per dispatch, derived
issue rates, and HBM-side bytes per k_verify_dsm launch (FETCH_SIZE x2, the
gfx950 correction in MI355X_MICROARCH.md, + WRITE_SIZE)."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]                      # gpurun_out/prof_<tag>
out = sys.argv[2]                    # profiles/<tag>_pmc_summary.json
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {"source": "rocprofv3 --pmc (one counter group per run) on: python3 bench.py --contexts 1 --no-c4 --no-cpu-baseline --steps 2 "
                 "--warmup 1; values are means per dispatch", "kernels": {}}
for k in ("k_verify_prep", "k_verify_dsm"):
    if k not in acc:
        continue
    m = {c: sum(v) / len(v) for c, v in acc[k].items()}
    der = {}
    if "SQ_INSTS_VALU" in m and "SQ_WAVES" in m:
        der["valu_instr_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
    if "SQ_INSTS_VALU_INT32" in m and "SQ_INSTS_VALU" in m:
        der["int32_valu_share"] = m["SQ_INSTS_VALU_INT32"] / m["SQ_INSTS_VALU"]
        der["int64_valu_share (v_mad_u64_u32, 64-bit shifts)"] = m.get("SQ_INSTS_VALU_INT64", 0) / m["SQ_INSTS_VALU"]
    if "SQ_WAVE_CYCLES" in m:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in m:
                der[c.lower() + "_frac_of_wave_cycles"] = m[c] / m["SQ_WAVE_CYCLES"]
    if "TCC_HIT_sum" in m:
        der["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
    if "FETCH_SIZE" in m:
        der["fetch_bytes_x2_corrected"] = 2 * m["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in m:
        der["write_bytes"] = m["WRITE_SIZE"] * 1024
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        der["hbm_side_bytes_per_launch"] = der["fetch_bytes_x2_corrected"] + der["write_bytes"]
    m["derived"] = der
    res["kernels"][k] = m
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd.kernel_hash import kernel_hashes  # noqa: E402  (the machine code these counters describe)
res["kernel_sha"] = kernel_hashes(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "firedancer_amd", "libfd_ed25519_hip.so"))
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v["derived"] for k, v in res["kernels"].items()}, indent=1))
