#!/bin/bash
# r03o: HEAD checkpoint -- full GPU suite, smoke, C2 and C4 bench lines
set -o pipefail
O=gpurun_out/r03o; mkdir -p $O
export FD_DROPIN_SUMMARY=$O/dropin_c_callers.json
timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -rP > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
grep -h "C callers\|concurrent drop-in\|16 threads" $O/pytest_gpu.txt | head -6
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
cut -c1-300 $O/bench_c2.json
timeout -k 10 400 python bench.py --config c4 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
cut -c1-300 $O/bench_c4.json
