#!/bin/bash
# r03ac: latency path, racing copies (default) vs calibrated pull (FD_ED25519_HIP_LAT_PULL=1):
# lone launches by size, drop-in C callers, latency/parity tests under pull
set -o pipefail
R=$PWD; O=$R/gpurun_out/r03ac; mkdir -p $O
FD_ED25519_HIP_LAT_PULL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_latency.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_pull.txt 2>&1 || { tail -30 $O/pytest_pull.txt; exit 1; }
tail -1 $O/pytest_pull.txt
timeout -k 10 120 python3 -c "import sys; sys.path.insert(0,'tests'); from test_gpu_dropin_concurrent import _harness_input; _harness_input('$O/calls.bin', 64, 12, 64, 0x1612)" || exit 1
for pull in 0 1; do
  FD_ED25519_HIP_LAT_PULL=$pull timeout -k 10 200 python3 tools/lat_copies.py 20 1,12,48,192 16 > $O/lone_$pull.txt 2>&1 || { tail -5 $O/lone_$pull.txt; exit 1; }
  echo "pull $pull"; grep "^n " $O/lone_$pull.txt
  for t in 1 16 64; do
    FD_ED25519_HIP_LAT_PULL=$pull timeout -k 10 60 $R/tools/dropin_threads $O/calls.bin 1.5 $t > $O/h_${pull}_t$t.json 2>> $O/err.txt || { echo fail; exit 1; }
    python3 -c "import json; d=json.load(open('$O/h_${pull}_t$t.json')); print('  pull $pull threads $t:', round(d['sigs_per_s']/1e6,3), 'M/s p50', d['p50_us'], 'p99', d['p99_us'], 'cpl', d['calls_per_launch'])"
  done
done
