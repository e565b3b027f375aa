#!/bin/bash
# r03j: product-build latency-path launch time vs racing copies, three processes
set -o pipefail
O=gpurun_out/r03j; mkdir -p $O
for p in 1 2 3; do
  timeout -k 10 120 python3 tools/lat_copies.py 40 > $O/p$p.txt 2>&1 || { tail -20 $O/p$p.txt; exit 1; }
  echo "== process $p"; grep "^n " $O/p$p.txt
done
