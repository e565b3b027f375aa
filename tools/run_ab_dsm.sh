#!/bin/bash
# GPU-box script: GPU tests on the default build, then C2 and C4 benches
# alternating the default build with library variants.
# Usage: bash tools/run_ab_dsm.sh <tag> <variant>...   (firedancer_amd/libfd_ed25519_hip_<variant>.so)
T=$1; shift; O=gpurun_out/ab_$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_default.log 2>&1 \
    || { echo "pytest failed"; tail -30 $O/pytest_default.log; exit 1; }
tail -1 $O/pytest_default.log
for rep in 1 2; do
  for v in default "$@"; do
    if [ $v != default ]; then export FD_ED25519_HIP_LIB=$PWD/firedancer_amd/libfd_ed25519_hip_$v.so; else unset FD_ED25519_HIP_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || { tail -5 $O/c2_${v}_$rep.err; exit 1; }
    timeout -k 10 400 python bench.py --config c4 --steps 8 --warmup 2 --no-cpu-baseline > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { tail -5 $O/c4_${v}_$rep.err; exit 1; }
    python3 -c "
import json; a=json.load(open('$O/c2_${v}_$rep.json')); b=json.load(open('$O/c4_${v}_$rep.json'))
print('$v', $rep, 'c2', round(a['value']/1e6,2), 'prep', a['pipeline']['prep_ms'], 'dsm', a['pipeline']['dsm_ms'], '| c4', round(b['value']/1e6,2), 'prep', b['roofline']['prep_ms_per_batch'], 'dsm', b['roofline']['avg_launch_ms'], 'pcie', round(b['pcie_inclusive']['value']/1e6,2))"
  done
done
