#!/bin/bash
# GPU-box script: bench one config for each verify-context count given, no
# CPU baseline.  Usage: CFG=c2 bash tools/run_contexts.sh 1 2 3 4
set -o pipefail
mkdir -p gpurun_out
for c in "$@"; do
  timeout -k 10 300 python bench.py --config ${CFG:-c2} --contexts $c --no-cpu-baseline --steps ${STEPS:-20} --warmup 2 > gpurun_out/bench_${CFG:-c2}_ctx$c.json 2> gpurun_out/bench_ctx$c.err || { tail -20 gpurun_out/bench_ctx$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${CFG:-c2}_ctx$c.json')); print('${CFG:-c2} contexts $c', d['value'], d['ms_per_step'], 'prep', d['pipeline']['prep_ms'], 'dsm', d['pipeline']['dsm_ms'], 'frac', d['roofline']['frac'])"
done
