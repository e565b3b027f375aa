#!/bin/bash
# C4 tile-count A/B on one box (resident leg only)
set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
for t in 6 4 8 12 6; do
  timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --c4-pcie-steps 1 --tiles $t > $O/c4_t$t.json 2> $O/c4_t$t.err || { tail -20 $O/c4_t$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4_t$t.json')); print('tiles $t', d['value'], d.get('batch_gpu_ms'), d.get('ms_per_step'))"
done
