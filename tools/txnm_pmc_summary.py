#!/usr/bin/env python3
"""Summarise the FETCH_SIZE / WRITE_SIZE passes of tools/gpu_session.sh's
c4pmc step (bench.py --config c4 --tiles 1: every k_txnm_batch<16> dispatch
is a whole 2^20-frag batch of the same stream) into
profiles/<tag>_c4_pmc_summary.json, the file bench.py's C4 ingest roofline
reads (PMC_SUMMARY_C4):

  hbm_side_bytes_per_launch    = FETCH_SIZE x 2 (gfx950: FETCH_SIZE counts
                                 wide coalesced reads at half their bytes,
                                 MI355X_MICROARCH.md HBM section) + WRITE_SIZE,
                                 both in KiB per dispatch in rocprofv3's output
  algorithmic_bytes_per_launch = the bench line's ingest_roofline bytes (the
                                 kernel's own byte count, fd_verify_hip.h)

Other access widths are uncalibrated (the kernel's 2-byte fd_txn_t stores and
single-lane header reads), so the ratio is an upper estimate of re-reads.
usage: python tools/txnm_pmc_summary.py gpurun_out/<tag> profiles/<tag>_c4_pmc_summary.json"""
import collections
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def per_dispatch(d, counter):
    """{dispatch id: (kernel name, value)} for one counter of one pass."""
    out = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] == counter:
            out[int(r["Dispatch_Id"])] = (r["Kernel_Name"], float(r["Counter_Value"]))
    return out


def main():
    d, out_path = sys.argv[1], sys.argv[2]
    res = {"source": f"{d}: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) --kernel-trace -- "
                     "bench.py --config c4 --tiles 1 --no-cpu-baseline --steps 2 --warmup 1 --c4-pcie-steps 1; "
                     "means over the full-batch dispatches", "kernels": {}}
    vals = collections.defaultdict(dict)
    for pas, ctr in (("c4pmc_fetch", "FETCH_SIZE"), ("c4pmc_write", "WRITE_SIZE")):
        by_k = collections.defaultdict(list)
        for _, (k, v) in sorted(per_dispatch(os.path.join(d, pas), ctr).items()):
            by_k[k.split("(")[0].replace("void ", "")].append(v)
        for k, vs in by_k.items():
            full = [v for v in vs if v >= 0.5 * max(vs)]          # whole batches (the warm-up frag is tiny)
            vals[k][ctr] = sum(full) / len(full)
            vals[k][ctr + "_dispatches"] = len(full)
    bench = json.loads([l for l in open(os.path.join(d, "c4pmc_fetch.out")) if l.startswith("{")][-1])
    ing = bench.get("ingest_roofline") or {}
    for k, m in vals.items():
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["hbm_side_bytes_per_launch"] = m["FETCH_SIZE"] * 1024 * 2 + m["WRITE_SIZE"] * 1024
        res["kernels"][k] = m
    kb = res["kernels"].get("k_txnm_batch<16>")
    if kb and ing.get("algorithmic_bytes_per_launch"):
        kb["algorithmic_bytes_per_launch"] = ing["algorithmic_bytes_per_launch"]
        kb["frags_per_launch"] = ing.get("frags_per_launch")
        kb["traffic_ratio"] = kb["hbm_side_bytes_per_launch"] / kb["algorithmic_bytes_per_launch"]
        res["kernels"]["k_txnm_batch"] = kb
    from firedancer_amd.kernel_hash import kernel_hashes
    res["kernel_sha"] = kernel_hashes(os.path.join(REPO, "firedancer_amd", "libfd_ed25519_hip.so"),
                                      ("k_verify_dsm", "k_verify_prep", "k_txnm_batch<16>"))
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res["kernels"].get("k_txnm_batch"), indent=1))


if __name__ == "__main__":
    main()
