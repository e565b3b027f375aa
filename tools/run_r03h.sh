#!/bin/bash
# r03h: is the lone k_verify_lat workgroup slow because the device idles at a low clock?
#  lat_trace alone, then with tools/heater.py keeping the GPU busy from another process; clocks sampled by rocm-smi
set -o pipefail
O=gpurun_out/r03h; mkdir -p $O
export FD_ED25519_HIP_LIB=$PWD/firedancer_amd/libfd_ed25519_hip_lattrace.so
rocm-smi --showperflevel --showclocks > $O/smi_idle.txt 2>&1
timeout -k 10 120 python3 tools/lat_trace.py 1 40 > $O/alone.txt 2>&1 || { tail -20 $O/alone.txt; exit 1; }
echo "== alone"; grep "^xcc [04]" $O/alone.txt
timeout -k 10 60 python3 tools/heater.py 30 > $O/heater.txt 2>&1 &
HP=$!
sleep 8
rocm-smi --showclocks > $O/smi_heated.txt 2>&1
timeout -k 10 120 python3 tools/lat_trace.py 1 40 > $O/heated.txt 2>&1 || { tail -20 $O/heated.txt; kill $HP; exit 1; }
rocm-smi --showclocks > $O/smi_heated2.txt 2>&1
echo "== with heater"; grep "^xcc [04]" $O/heated.txt
wait $HP
timeout -k 10 120 python3 tools/lat_trace.py 1 40 > $O/after.txt 2>&1 || { tail -20 $O/after.txt; exit 1; }
echo "== after"; grep "^xcc [04]" $O/after.txt
grep -i "sclk\|perf" $O/smi_idle.txt $O/smi_heated.txt $O/smi_heated2.txt | head -20
