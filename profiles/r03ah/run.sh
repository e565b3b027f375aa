#!/bin/bash
# r03ah: C2 by context count (independent chunk pipelines) on the 4-wave prep build
set -o pipefail
O=gpurun_out/r03ah; mkdir -p $O
for rep in 1 2; do
  for c in 1 2 3 4; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --contexts $c > $O/c2_ctx${c}_$rep.json 2> $O/c2_ctx${c}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$O/c2_ctx${c}_$rep.json')); print('contexts $c rep $rep', round(d['value']/1e6,2), 'ms/step', d['ms_per_step'])"
  done
done
