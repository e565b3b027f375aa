#!/usr/bin/env python3
"""Summarise tools/run_c4_issue.sh into profiles/<tag>_c4_valu_issue.json.

The last k_verify_dsm dispatch of bench.py --config c4 is the timing leg's
tile-0 batch, whose survivor count the bench line reports as
roofline.units_per_launch; its counters give C4's own issue slots and cycles
per launch (same definitions as tools/valu_calib_summary.py).  bench.py reads
this file for C4 (slots_scaled_from_c2 false when the unit counts agree).
usage: python tools/c4_issue_summary.py gpurun_out/c4issue_<tag> profiles/<tag>_c4_valu_issue.json"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from valu_calib_summary import derive, load  # noqa: E402


def main():
    d, out = sys.argv[1], sys.argv[2]
    eng = load(os.path.join(d, "engine"))
    bench = json.loads([l for l in open(os.path.join(d, "bench.json")) if l.startswith("{")][-1])
    units = bench["roofline"]["units_per_launch"]
    res = {"source": f"{d}: rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU "
                     "SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_BUSY_CYCLES SQ_WAVES "
                     "GRBM_GUI_ACTIVE GRBM_COUNT (one pass) --kernel-trace -- bench.py --config c4 --steps 2 "
                     "--warmup 1 --c4-pcie-steps 1; the last dispatch of each kernel (the timing leg's tile-0 batch)",
           "definition": "issue slots = SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2; slot_util = slots / "
                         "(1024 SIMDs x GRBM_GUI_ACTIVE/8 / 4)",
           "engine": {}}
    for k in ("k_verify_prep", "k_verify_dsm"):
        xs = sorted((int(i), x) for i, x in eng.items() if x["kernel"] == k)
        if xs:
            r = {kk: round(v, 4 if kk != "valu_insts" else 0) for kk, v in derive(xs[-1][1]).items()}
            r["dispatches_in_run"] = len(xs)
            res["engine"][k] = r
    res["engine"]["k_verify_dsm"]["units"] = units
    from firedancer_amd.kernel_hash import kernel_hashes
    res["kernel_sha"] = kernel_hashes(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                   "firedancer_amd", "libfd_ed25519_hip.so"))
    res["bench_value"] = bench["value"]
    cal = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                                      os.environ.get("FD_ISSUE_CALIBRATION", "r03ag_valu_issue_calibration.json"))))
    res["single_issue_ceiling_slot_util"] = cal.get("single_issue_ceiling_slot_util")   # same microbenchmark
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["engine"], indent=1))


if __name__ == "__main__":
    main()
