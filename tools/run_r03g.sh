#!/bin/bash
# r03g: per-XCD phase timing of lone k_verify_lat workgroups (diagnostic build), three processes
set -o pipefail
O=gpurun_out/r03g; mkdir -p $O
export FD_ED25519_HIP_LIB=$PWD/firedancer_amd/libfd_ed25519_hip_lattrace.so
for p in 1 2 3; do
  timeout -k 10 120 python3 tools/lat_trace.py 1 40 > $O/trace_n1_p$p.txt 2>&1 || { tail -20 $O/trace_n1_p$p.txt; exit 1; }
  echo "== process $p (n=1)"; grep "^xcc 0\|^working" $O/trace_n1_p$p.txt
done
timeout -k 10 120 python3 tools/lat_trace.py 12 20 > $O/trace_n12.txt 2>&1 || { tail -20 $O/trace_n12.txt; exit 1; }
echo "== n=12"; grep "^xcc 0\|^working" $O/trace_n12.txt
