#!/bin/bash
# round-4 session s: the full GPU suite, smoke, and the default bench line (C2 + c4 + tile legs)
set -o pipefail
O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
t0=$(date +%s%N)
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
t1=$(date +%s%N); echo "bench wall_s $(( (t1-t0)/1000000000 ))" | tee $O/bench_wall.txt
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('c2', d['value'], 'c4', d['c4']['value'], 'tile', json.dumps(d.get('tile'))[:600])"
