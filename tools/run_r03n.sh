#!/bin/bash
# r03n: k_verify_lat workgroup size 768 / 512 / 256 threads (1 / 2 / 4 per CU), copy budget in
# workgroup slots split over 4 drop-in slots: C callers (1/16/64 threads x 12 sigs) and lone launches
set -o pipefail
R=$PWD; O=$R/gpurun_out/r03n; mkdir -p $O
timeout -k 10 120 python3 -c "import sys; sys.path.insert(0,'tests'); from test_gpu_dropin_concurrent import _harness_input; _harness_input('$O/calls.bin', 64, 12, 64, 0x1612)" || exit 1
for v in d768 wg512 wg256; do
  LP=""; LIB=""
  if [ $v != d768 ]; then mkdir -p $O/v_$v && ln -sf $R/firedancer_amd/libfd_ed25519_hip_$v.so $O/v_$v/libfd_ed25519_hip.so; LP=$O/v_$v; LIB=$R/firedancer_amd/libfd_ed25519_hip_$v.so; fi
  for rep in 1 2; do for t in 1 16 64; do
    LD_LIBRARY_PATH=$LP timeout -k 10 60 $R/tools/dropin_threads $O/calls.bin 1.5 $t > $O/${v}_t${t}_$rep.json 2>> $O/err.txt || { echo "fail $v"; tail -3 $O/err.txt; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${v}_t${t}_$rep.json')); print('$v threads $t rep $rep:', round(d['sigs_per_s']/1e6,3), 'M/s p50', d['p50_us'], 'p99', d['p99_us'], 'cpl', d['calls_per_launch'])"
  done; done
  FD_ED25519_HIP_LIB=$LIB timeout -k 10 120 python3 tools/lat_copies.py 20 1,12,32 1,8 > $O/${v}_lone.txt 2>&1 || { tail -5 $O/${v}_lone.txt; exit 1; }
  grep "^n " $O/${v}_lone.txt
done
