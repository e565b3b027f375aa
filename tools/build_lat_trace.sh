#!/bin/bash
# Build the latency-kernel trace library (diagnostic, never the product):
# applies tools/lat_trace.patch (s_memrealtime at every phase boundary, HW_ID
# per working wave, racing copies run to completion) to a scratch copy of the
# sources and writes firedancer_amd/libfd_ed25519_hip_lattrace.so for
# tools/lat_trace.py (FD_ED25519_HIP_LIB=...).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/firedancer_amd $T/include
cp -r $R/firedancer_amd/csrc $T/firedancer_amd/csrc && cp $R/include/*.h $T/include/
(cd $T && patch -s -p0 < $R/tools/lat_trace.patch)
C=$T/firedancer_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -DFD_LAT_TRACE=1 \
  -o $R/firedancer_amd/libfd_ed25519_hip_lattrace.so $C/fd_ed25519_hip.hip $C/fd_txn_hip.hip $C/fd_sha512_hip.hip
rm -rf $T
