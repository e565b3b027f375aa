#!/bin/bash
# r03ae: prep register pressure -- HEAD (158 VGPRs) vs prefix/S loads moved
# out of the live range (132, default build) vs the same at 4 waves/SIMD
# (128 + 10 spills): parity subset per build, then C2 and C4 alternating
set -o pipefail
O=gpurun_out/r03ae; mkdir -p $O
V="firedancer_amd/libfd_ed25519_hip_head.so firedancer_amd/libfd_ed25519_hip.so firedancer_amd/libfd_ed25519_hip_prep4.so"
for v in $V; do
  n=$(basename $v .so)
  FD_ED25519_HIP_LIB=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
      tests/test_sha512_cavp.py tests/test_gpu_sha512.py tests/test_gpu_txnm.py -m gpu > $O/pytest_$n.log 2>&1 || { echo "pytest $n failed"; tail -20 $O/pytest_$n.log; exit 1; }
  echo "$n $(tail -1 $O/pytest_$n.log)"
done
for rep in 1 2; do
  for v in $V; do
    n=$(basename $v .so)
    FD_ED25519_HIP_LIB=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_${n}_$rep.json 2> $O/c2_${n}_$rep.err || exit 1
    FD_ED25519_HIP_LIB=$v timeout -k 10 400 python bench.py --config c4 --steps 8 --warmup 2 --no-cpu-baseline > $O/c4_${n}_$rep.json 2> $O/c4_${n}_$rep.err || exit 1
    python3 -c "
import json; a=json.load(open('$O/c2_${n}_$rep.json')); b=json.load(open('$O/c4_${n}_$rep.json'))
print('$n', $rep, 'c2', round(a['value']/1e6,2), 'prep', a['pipeline']['prep_ms'], 'c4', round(b['value']/1e6,2), 'c4 prep', b['roofline']['prep_ms_per_batch'])"
  done
done
