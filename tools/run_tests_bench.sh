#!/bin/bash
# GPU-box script: parity tests, then bench (stop on the first failure).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/pytest_gpu.log; exit $rc; fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
