#!/usr/bin/env python3
"""Summarise tools/run_profile_c4.sh output into profiles/<tag>_c4_pmc_summary.json:
per-kernel means per dispatch (one dispatch = one tile batch), and k_verify_prep's
ingest against the algorithmic bytes with the gfx950 FETCH_SIZE calibration of
profiles/r02h_fetch_calibration (per-record 16-B loads at a 64-B stride count
0.914x their bytes; wave-cooperative 16-B message pieces 0.516x).
usage: python tools/c4_pmc_summary.py gpurun_out/prof_c4_<tag> profiles/<tag>_c4_pmc_summary.json"""
import collections
import csv
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def algorithmic(txns=1 << 20, tiles=2, seed=0x5eed0004):
    """Records and message bytes of tile 0's batch of the bench's C4 stream
    (the stream's shape does not depend on the signatures)."""
    from firedancer_amd.txn_workload import make_txn_stream
    s = make_txn_stream(txns, lambda p, *_: (np.zeros((p.shape[0], 32), np.uint8), np.zeros((p.shape[0], 64), np.uint8)),
                        seed=seed)
    sel = np.arange(0, s.n, tiles)
    sz = s.sz[sel].astype(np.int64); nsig = s.nsig[sel].astype(np.int64)
    msg = sz - 1 - 64 * nsig
    ok = (msg > 0) & (nsig >= 1) & (nsig <= 16)
    return int(nsig[ok].sum()), int(msg[ok].sum()), int((nsig[ok] * msg[ok]).sum())


def main():
    d, out_path = sys.argv[1], sys.argv[2]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for i in range(1, 5):
        for r in csv.DictReader(open(os.path.join(d, f"p{i}", "run_counter_collection.csv"))):
            acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"source": f"{d}: rocprofv3 --pmc passes of bench.py --config c4 --steps 3 --warmup 1; means per dispatch",
           "kernels": {}}
    for k, m0 in acc.items():
        m = {c: sum(v) / len(v) for c, v in m0.items()}
        der = {}
        if "FETCH_SIZE" in m:
            der["fetch_size_raw_bytes"] = m["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in m:
            der["write_bytes"] = m["WRITE_SIZE"] * 1024
        if "SQ_INSTS_VALU" in m:
            der["issue_slot_util"] = (m["SQ_INSTS_VALU"] - m["SQ_ACTIVE_INST_VALU2"]) / (1024 * m["GRBM_GUI_ACTIVE"] / 32)
            der["vmem_rd_per_wave"] = m["SQ_INSTS_VMEM_RD"] / m["SQ_WAVES"]
            der["lds_instr_per_wave"] = m["SQ_INSTS_LDS"] / m["SQ_WAVES"]
        if "TCC_HIT_sum" in m:
            der["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        m["derived"] = der
        out["kernels"][k] = m
    recs, uniq, perrec = algorithmic()
    raw = out["kernels"]["k_verify_prep"]["derived"]["fetch_size_raw_bytes"]
    rec_true = recs * 104
    est = rec_true + (raw - rec_true * 0.914) / 0.516
    out["prep_ingest_c4"] = {
        "records_per_dispatch": recs, "unique_message_bytes": uniq, "per_record_message_bytes": perrec,
        "algorithmic_bytes_unique_messages": recs * 104 + uniq,
        "algorithmic_bytes_per_record_messages": recs * 104 + perrec,
        "fetch_raw_bytes": raw, "estimated_true_fetch_bytes": est,
        "ratio_vs_unique": est / (recs * 104 + uniq), "ratio_vs_per_record": est / (recs * 104 + perrec)}
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps(out["prep_ingest_c4"], indent=1))


if __name__ == "__main__":
    main()
