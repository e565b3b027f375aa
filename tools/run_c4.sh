#!/bin/bash
# GPU-box script: verify-tile GPU tests, then a short C4 bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_txn.py -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu_txn.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu_txn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --config c4 --steps 5 --warmup 1 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -30 gpurun_out/bench_c4.err; exit 1; }
cat gpurun_out/bench_c4.json
