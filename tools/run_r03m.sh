#!/bin/bash
# r03m: drop-in C callers (16 and 64 threads x 12 signatures): batch slots, latency-kernel
# workgroup size (768 default / 256 variant) and per-slot copy budget
set -o pipefail
R=$PWD; O=$R/gpurun_out/r03m; mkdir -p $O
timeout -k 10 120 python3 -c "import sys; sys.path.insert(0,'tests'); from test_gpu_dropin_concurrent import _harness_input; _harness_input('$O/calls.bin', 64, 12, 64, 0x1612)" || exit 1
mkdir -p $O/v_wg256 && ln -sf $R/firedancer_amd/libfd_ed25519_hip_wg256.so $O/v_wg256/libfd_ed25519_hip.so
run() {  # tag libdir slots latcus threads
  LD_LIBRARY_PATH=$2 FD_ED25519_HIP_DROPIN_SLOTS=$3 FD_ED25519_HIP_DROPIN_LAT_CUS=$4 timeout -k 10 60 $R/tools/dropin_threads $O/calls.bin 1.5 $5 > $O/$1_s$3_c$4_t$5.json 2>> $O/err.txt || { echo "fail $1"; tail -3 $O/err.txt; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1_s$3_c$4_t$5.json')); print('$1 slots $3 latcus $4 threads $5:', round(d['sigs_per_s']/1e6,3), 'M/s p50', d['p50_us'], 'p99', d['p99_us'], 'cpl', d['calls_per_launch'])"
}
for t in 16 64; do
  run d768 "" 4 64 $t || exit 1
  run d768 "" 8 32 $t || exit 1
  run d768 "" 16 16 $t || exit 1
  run w256 $O/v_wg256 4 256 $t || exit 1
  run w256 $O/v_wg256 8 128 $t || exit 1
  run w256 $O/v_wg256 16 64 $t || exit 1
  run w256 $O/v_wg256 16 96 $t || exit 1
done
