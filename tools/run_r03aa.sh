#!/bin/bash
# r03aa: racing-copy cap 8 (one per XCD) vs 12 / 16: lone calls (tools/lat_copies.py) and C callers
set -o pipefail
R=$PWD; O=$R/gpurun_out/r03aa; mkdir -p $O
timeout -k 10 120 python3 -c "import sys; sys.path.insert(0,'tests'); from test_gpu_dropin_concurrent import _harness_input; _harness_input('$O/calls.bin', 64, 12, 64, 0x1612)" || exit 1
for cap in 8 16 12; do
  FD_ED25519_HIP_LAT_COPIES=$cap timeout -k 10 200 python3 tools/lat_copies.py 30 1,12,16,32 32 > $O/lone_$cap.txt 2>&1 || { tail -5 $O/lone_$cap.txt; exit 1; }
  echo "cap $cap"; grep "^n " $O/lone_$cap.txt
  for t in 1 16; do
    FD_ED25519_HIP_LAT_COPIES=$cap timeout -k 10 60 $R/tools/dropin_threads $O/calls.bin 1.5 $t > $O/h_${cap}_t$t.json 2>> $O/err.txt || { echo fail; exit 1; }
    python3 -c "import json; d=json.load(open('$O/h_${cap}_t$t.json')); print('  cap $cap threads $t:', round(d['sigs_per_s']/1e6,3), 'M/s p50', d['p50_us'], 'p99', d['p99_us'])"
  done
done
