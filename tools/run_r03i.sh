#!/bin/bash
# r03i: the shader clock of lone k_verify_lat launches, from PMC (GRBM_GUI_ACTIVE cycles over the
# dispatch's own duration), in three processes of the diagnostic build (8 full copies per launch)
set -o pipefail
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03i; mkdir -p $O
export FD_ED25519_HIP_LIB=$R/firedancer_amd/libfd_ed25519_hip_lattrace.so
G="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
for p in 1 2 3; do
  timeout -s KILL 100 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/p$p -o run -- python3 tools/lat_trace.py 1 30 > $O/p$p.txt 2> $O/p$p.err
  echo "p$p rc=$?"; grep "^xcc [0]" $O/p$p.txt
  python3 - $O/p$p <<'PY'
import csv, glob, sys, collections
import numpy as np
cnt = collections.defaultdict(dict); dur = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("k_verify_lat"):
            cnt[int(r["Dispatch_Id"])][r["Counter_Name"]] = cnt[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("k_verify_lat"):
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
ghz = []; us = []
for d, c in cnt.items():
    if d in dur and c.get("GRBM_GUI_ACTIVE"):
        ghz.append(c["GRBM_GUI_ACTIVE"] / 8 / (dur[d] * 1e3)); us.append(dur[d])
print("  dispatches", len(us), "us p50", round(float(np.median(us)), 1), "GRBM clock GHz p10/50/90", np.percentile(ghz, [10, 50, 90]).round(3),
      "ipc", round(float(np.median([c["SQ_INSTS_VALU"] / max(c["SQ_BUSY_CYCLES"], 1) for c in cnt.values()])), 4))
PY
done
