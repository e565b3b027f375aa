#!/bin/bash
# round 5 session q: cores for the GPU tile process (HIP runtime threads), more outstanding work per tile
out=gpurun_out/r05q; mkdir -p $out
export TMPDIR=/tmp
run() { # name tiles run-env cores
  SVC_BENCH_SVC_CORES=$4 timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "$3" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
run c1 2,3 "SVC_RUN_REQ_DEPTH=8" 1 || exit $?
run c3 2,3 "SVC_RUN_REQ_DEPTH=8" 3 || exit $?
run c6 2,3 "SVC_RUN_REQ_DEPTH=8" 6 || exit $?
run c3d16 2,3 "SVC_RUN_REQ_DEPTH=16" 3 || exit $?
run c3d24 2 "SVC_RUN_REQ_DEPTH=24" 3 || exit $?
SVC_BENCH_SVC_CORES=3 timeout -k 10 240 python -u tools/svc_bench.py --frags 4194304 --tiles 2 --prelay --env SVC_RUN_REQ_DEPTH=8 \
  --rocprof $out/prof --timeout 200 --logdir $out/logsp > $out/prof.jsonl 2> $out/prof.err || exit $?
python3 tools/trace_util.py $out/prof/t2_0 > $out/util_t2.json
find $out/prof -name "*trace*.csv" -delete
