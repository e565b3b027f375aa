#!/bin/bash
# r03w: drop-in ring with per-block condition variables: concurrency tests + C callers (3 reps)
set -o pipefail
R=$PWD; O=$R/gpurun_out/r03w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin_concurrent.py tests/test_gpu_parity.py -m gpu -v -s --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
grep -h "passed\|C callers\|concurrent drop-in" $O/pytest.txt
timeout -k 10 120 python3 -c "import sys; sys.path.insert(0,'tests'); from test_gpu_dropin_concurrent import _harness_input; _harness_input('$O/calls.bin', 64, 12, 64, 0x1612)" || exit 1
for rep in 1 2 3; do for t in 16 64; do
  timeout -k 10 60 $R/tools/dropin_threads $O/calls.bin 1.5 $t > $O/t${t}_$rep.json 2>> $O/err.txt || { echo fail; exit 1; }
  python3 -c "import json; d=json.load(open('$O/t${t}_$rep.json')); print('threads $t rep $rep:', round(d['sigs_per_s']/1e6,3), 'M/s p50', d['p50_us'], 'p99', d['p99_us'], 'cpl', d['calls_per_launch'])"
done; done
