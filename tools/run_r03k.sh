#!/bin/bash
# r03k: raw per-workgroup phase timing + hardware ids of lone k_verify_lat workgroups (diagnostic build)
set -o pipefail
O=gpurun_out/r03k; mkdir -p $O
export FD_ED25519_HIP_LIB=$PWD/firedancer_amd/libfd_ed25519_hip_lattrace.so
for p in 1 2; do
  FD_LAT_TRACE_RAW=$O/raw_p$p.json timeout -k 10 120 python3 tools/lat_trace.py 1 60 > $O/p$p.txt 2>&1 || { tail -20 $O/p$p.txt; exit 1; }
  grep "^working" $O/p$p.txt
done
