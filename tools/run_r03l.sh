#!/bin/bash
# r03l: latency-path launch time vs batch size and racing copies, k_verify_lat workgroups of
# 768 threads (one per CU, default) vs 256 (up to four per CU)
set -o pipefail
O=gpurun_out/r03l; mkdir -p $O
for v in cp256 wg256; do
  if [ $v = default ]; then unset FD_ED25519_HIP_LIB; else export FD_ED25519_HIP_LIB=$PWD/firedancer_amd/libfd_ed25519_hip_$v.so; fi
  timeout -k 10 200 python3 tools/lat_copies.py 20 1,12,48,96,192 1,2,4,8 > $O/$v.txt 2>&1 || { tail -20 $O/$v.txt; exit 1; }
  echo "== $v"; grep "^n " $O/$v.txt
done
