#!/bin/bash
# r03af: k_verify_prep at 3 waves/SIMD (132 VGPRs) vs 4 (128 + 10 spills): C2 and C4, 4 alternating reps
set -o pipefail
O=gpurun_out/r03af; mkdir -p $O
V="firedancer_amd/libfd_ed25519_hip.so firedancer_amd/libfd_ed25519_hip_prep4.so"
for rep in 1 2 3 4; do
  for v in $V; do
    n=$(basename $v .so)
    FD_ED25519_HIP_LIB=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_${n}_$rep.json 2> $O/c2_${n}_$rep.err || exit 1
    FD_ED25519_HIP_LIB=$v timeout -k 10 400 python bench.py --config c4 --steps 8 --warmup 2 --no-cpu-baseline > $O/c4_${n}_$rep.json 2> $O/c4_${n}_$rep.err || exit 1
    python3 -c "
import json; a=json.load(open('$O/c2_${n}_$rep.json')); b=json.load(open('$O/c4_${n}_$rep.json'))
print('$n', $rep, 'c2', round(a['value']/1e6,2), 'prep', a['pipeline']['prep_ms'], 'c4', round(b['value']/1e6,2), 'c4 prep', b['roofline']['prep_ms_per_batch'])"
  done
done
