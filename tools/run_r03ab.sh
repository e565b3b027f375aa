#!/bin/bash
# r03ab: copy policy on HEAD (up to 16 racing copies, one workgroup per CU): latency/drop-in/parity tests,
# lone-call latency, C callers
set -o pipefail
R=$PWD; O=$R/gpurun_out/r03ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_latency.py tests/test_gpu_dropin_concurrent.py tests/test_gpu_parity.py tests/test_gpu_streams.py -m gpu -v -s --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
grep -h "passed\|failed\|C callers" $O/pytest.txt
timeout -k 10 300 python3 tools/bench_latency.py 500 > $O/dropin_latency.json 2> $O/err.txt || { tail -10 $O/err.txt; exit 1; }
cat $O/dropin_latency.json
