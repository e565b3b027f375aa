#!/bin/bash
# r03x: lone latency-kernel time per CU (stream CU masks), two processes
set -o pipefail
O=gpurun_out/r03x; mkdir -p $O
for p in 1 2; do
  timeout -k 10 200 python3 -u tools/cu_latency.py 6 > $O/cu_p$p.txt 2>&1 || { tail -20 $O/cu_p$p.txt; exit 1; }
  tail -1 $O/cu_p$p.txt | python3 -c "import json,sys; d=json.load(sys.stdin); print('process $p always fast:', len(d['always_fast']), d['always_fast'][:64])"
done
