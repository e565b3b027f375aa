#!/bin/bash
# GPU-box script: C4 resident + PCIe-inclusive legs over verify-tile counts.
# Usage: bash tools/run_c4_pcie.sh <tag> <tiles>...
T=$1; shift; O=gpurun_out/c4pcie_$T; mkdir -p $O
for tiles in "$@"; do
  timeout -k 10 400 python3 bench.py --config c4 --steps 8 --warmup 2 --tiles $tiles --no-cpu-baseline \
      > $O/t$tiles.json 2> $O/t$tiles.err || exit $?
  python3 -c "import json; d=json.load(open('$O/t$tiles.json')); p=d['pcie_inclusive']; print('tiles $tiles', round(d['value']/1e6,2), 'pcie', round(p['value']/1e6,2), p['h2d_GBps'], p['results_equal_resident_leg'])"
done
