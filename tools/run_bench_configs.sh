#!/bin/bash
# GPU-box script: bench configs c1-c5 + a 1-process torch.distributed run (exercises the RCCL path).
set -o pipefail
O=gpurun_out/${1:-configs}; mkdir -p $O
for c in c2 c1 c3; do
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  cat $O/bench_$c.json
done
timeout -k 10 900 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
timeout -k 10 900 python bench.py --config c4 --steps 5 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
cat $O/bench_c4.json
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --no-cpu-baseline --force-dist > $O/bench_dist1.json 2> $O/bench_dist1.err || { tail -20 $O/bench_dist1.err; exit 1; }
cat $O/bench_dist1.json
