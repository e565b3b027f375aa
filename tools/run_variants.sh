#!/bin/bash
# GPU-box script: parity tests on the default library, then a short bench
# (no CPU baseline) for the default library and each named variant
# (firedancer_amd/libfd_ed25519_hip_<name>.so via FD_ED25519_HIP_LIB).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/pytest_gpu.log; exit $rc; fi
for v in default "$@"; do
  if [ "$v" = default ]; then lib=""; else lib="$PWD/firedancer_amd/libfd_ed25519_hip_$v.so"; fi
  FD_ED25519_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || { tail -20 gpurun_out/bench_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_$v.json')); print('$v', d['value'], 'prep', d['pipeline']['prep_ms'], 'dsm', d['pipeline']['dsm_ms'], 'frac', d['roofline']['frac'])"
done
