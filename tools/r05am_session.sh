#!/bin/bash
# round 5 session am: full GPU suite, smoke, the default bench line, a kernel profile of the bench's C2/C4 legs
out=gpurun_out/r05am; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_bench -o bench -- python3 bench.py --no-tile --no-cpu-baseline > $out/bench_prof.json 2> $out/bench_prof.err
find $out/prof_bench -name "*trace*.csv" -delete
