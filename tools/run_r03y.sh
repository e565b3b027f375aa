#!/bin/bash
# r03y: C4 GPU time per batch against tile count (1 tile = one launch sequence per 2^20-frag step)
set -o pipefail
O=gpurun_out/r03y; mkdir -p $O
for t in 1 2 6; do
  timeout -k 10 400 python bench.py --config c4 --tiles $t --steps 6 --warmup 2 --no-cpu-baseline --c4-pcie-steps 2 > $O/c4_t$t.json 2> $O/c4_t$t.err || { tail -5 $O/c4_t$t.err; exit 1; }
  python3 -c "
import json; b=json.load(open('$O/c4_t$t.json')); r=b['roofline']
print('tiles $t: c4', round(b['value']/1e6,2), 'ms/step', b['ms_per_step'], 'batch gpu ms', b['batch_gpu_ms'], 'host ms', b['batch_host_ms'], 'prep ms', r.get('prep_ms_per_batch'), 'dsm ms', r.get('avg_launch_ms'), 'launches', r.get('launches_per_batch'))"
done
