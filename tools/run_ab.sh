#!/bin/bash
# GPU-box script: A/B of build variants on the default bench (C2) and a parity
# subset.  Usage: bash tools/run_ab.sh <tag> <variant>...   ("" = default build)
T=$1; shift; O=gpurun_out/ab_$T; mkdir -p $O
for v in "$@"; do
  if [ -n "$v" ]; then export FD_ED25519_HIP_LIB=$v; else unset FD_ED25519_HIP_LIB; fi
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
      tests/test_gpu_halfsize.py -m gpu > $O/pytest_${v:-default}.log 2>&1 || { echo "pytest ${v:-default} failed"; tail -20 $O/pytest_${v:-default}.log; exit 1; }
  tail -1 $O/pytest_${v:-default}.log
done
for rep in 1 2; do
  for v in "$@"; do
    if [ -n "$v" ]; then export FD_ED25519_HIP_LIB=$v; else unset FD_ED25519_HIP_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_${v:-default}_$rep.json 2> $O/bench_${v:-default}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$O/bench_${v:-default}_$rep.json')); r=d['roofline']; print('${v:-default}', $rep, round(d['value']/1e6,2), 'dsm', r.get('avg_launch_ms'), 'prep', r.get('prep_ms_per_launch', r.get('prep_avg_ms')))"
  done
done
