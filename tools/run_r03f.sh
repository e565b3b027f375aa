#!/bin/bash
# r03f: drop-in call latency -- kernel time vs host time.
#  (1) kernel durations of k_verify_lat under --kernel-trace (default build, slots 1/4, threads 1/16)
#  (2) C-caller A/B: blocking hipStreamSynchronize (default) vs spin on hipStreamQuery (FD_DROPIN_SPIN=1), 3 processes each
set -o pipefail
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03f; mkdir -p $O
timeout -k 10 120 python3 -c "import sys; sys.path.insert(0,'tests'); from test_gpu_dropin_concurrent import _harness_input; _harness_input('$O/calls.bin', 64, 12, 64, 0x1612)" || exit 1
for sl in 1 4; do for th in 1 16; do
  FD_ED25519_HIP_DROPIN_SLOTS=$sl timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv -d $O/kt_s${sl}_t${th} -o run -- \
      $R/tools/dropin_threads $O/calls.bin 1 $th > $O/kt_s${sl}_t${th}.json 2> $O/kt_s${sl}_t${th}.err || { echo "kt $sl $th failed"; tail -5 $O/kt_s${sl}_t${th}.err; exit 1; }
  python3 - $O/kt_s${sl}_t${th} $O/kt_s${sl}_t${th}.json <<'PY'
import csv, glob, json, sys
import numpy as np
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
lat = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if r["Kernel_Name"].startswith("k_verify_lat")])
cp = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "copyBuffer" in r["Kernel_Name"]])
d = json.load(open(sys.argv[2]))
print(sys.argv[1].split("/")[-1], "calls p50", d["p50_us"], "| k_verify_lat n", lat.size, "p10/50/90", np.percentile(lat, [10, 50, 90]).round(1),
      "| copy kernels n", cp.size, "p50", round(float(np.median(cp)), 1) if cp.size else None)
PY
done; done
mkdir -p $O/v_spin && ln -sf $R/firedancer_amd/libfd_ed25519_hip_spin.so $O/v_spin/libfd_ed25519_hip.so
for rep in 1 2 3; do
  for v in default spin; do
    LP=""; [ $v = spin ] && LP=$O/v_spin
    for sl in 1 4; do for th in 1 16 64; do
      LD_LIBRARY_PATH=$LP FD_ED25519_HIP_DROPIN_SLOTS=$sl timeout -k 10 60 $R/tools/dropin_threads $O/calls.bin 1.5 $th > $O/h_${v}_s${sl}_t${th}_$rep.json 2>> $O/h_err.txt || { echo "harness $v failed"; tail -5 $O/h_err.txt; exit 1; }
      python3 -c "import json; d=json.load(open('$O/h_${v}_s${sl}_t${th}_$rep.json')); print('$v s$sl t$th r$rep', round(d['sigs_per_s']/1e6,3), 'M/s p50', d['p50_us'], 'p99', d['p99_us'], 'cpl', d['calls_per_launch'])"
    done; done
  done
done
