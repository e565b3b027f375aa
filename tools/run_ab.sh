#!/bin/bash
# GPU-box script: alternate C2 benches over named library variants (no tests):
#   bash tools/run_ab.sh default head default head
# variant "default" = firedancer_amd/libfd_ed25519_hip.so, else libfd_ed25519_hip_<name>.so
set -o pipefail
mkdir -p gpurun_out
i=0
for v in "$@"; do
  i=$((i+1))
  if [ "$v" = default ]; then lib=""; else lib="$PWD/firedancer_amd/libfd_ed25519_hip_$v.so"; fi
  FD_ED25519_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { tail -20 gpurun_out/ab_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$i.json')); p = d.get('pipeline') or {}; print('$v', d['value'], 'prep', p.get('prep_ms'), 'dsm', p.get('dsm_ms', d['roofline']['avg_launch_ms']))"
done
