#!/bin/bash
# GPU-box script: one bench line per argument set (no CPU baseline); prints
# value, DSM units per launch, DSM ms and units per ms.
#   bash tools/run_sweep.sh "--config c2" "--config c1 --sigs 933888" ...
set -o pipefail
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline $a > gpurun_out/sweep_$i.json 2> gpurun_out/sweep_$i.err || { tail -20 gpurun_out/sweep_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sweep_$i.json')); r=d['roofline']; print('$a', d['value'], r['units_per_launch'], r['avg_launch_ms'], round(r['units_per_launch']/r['avg_launch_ms']))"
done
