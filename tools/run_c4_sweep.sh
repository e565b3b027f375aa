#!/bin/bash
# GPU-box script: C4 verify-tile bench over tile counts / batch sizes.
# Usage: bash tools/run_c4_sweep.sh <tag> "<tiles list>" "<txns list>"
T=${1:-r02}; TL=${2:-"4 8"}; XL=${3:-"524288"}
mkdir -p gpurun_out/c4sweep_$T
for x in $XL; do for t in $TL; do
  timeout -k 10 300 python bench.py --config c4 --tiles $t --txns $x --steps 8 --warmup 2 --no-cpu-baseline \
      > gpurun_out/c4sweep_$T/t${t}_x${x}.json 2> gpurun_out/c4sweep_$T/t${t}_x${x}.err || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/c4sweep_$T/t${t}_x${x}.json')); print('tiles', $t, 'txns', $x, round(d['value']/1e6,2), 'M/s', d['ms_per_step'], 'ms', 'gpu', d['batch_gpu_ms'], 'host', d['batch_host_ms'])"
done; done
