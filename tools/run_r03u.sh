#!/bin/bash
# r03u: C4 (6 verify tiles, resident + PCIe legs) against the process's HIP hardware queue count
set -o pipefail
O=gpurun_out/r03u; mkdir -p $O
for rep in 1 2; do
  for q in 4 8 6; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > $O/c4_q${q}_$rep.json 2> $O/c4_q${q}_$rep.err || { tail -5 $O/c4_q${q}_$rep.err; exit 1; }
    python3 -c "
import json; b=json.load(open('$O/c4_q${q}_$rep.json'))
print('queues $q rep $rep: c4', round(b['value']/1e6,2), 'pcie', round(b['pcie_inclusive']['value']/1e6,2), 'batch gpu ms', b['batch_gpu_ms'])"
  done
done
