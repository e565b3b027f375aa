#!/bin/bash
# round 5 session j: merge policy with early ingest -- fewer, larger verify launches
out=gpurun_out/r05j; mkdir -p $out
export TMPDIR=/tmp
run() { # name svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles 2,3 --repeat 2 --prelay --env SVC_RUN_REQ_DEPTH=8 \
    --svc-env "$2" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
run base "SVC_MERGE_WAIT_NS=400000" || exit $?
run w2i2 "SVC_MERGE_WAIT_NS=2000000,SVC_INFLIGHT=2" || exit $?
run w2i2b "SVC_MERGE_WAIT_NS=2000000,SVC_INFLIGHT=2,SVC_BATCH_MAX=393216,SVC_MERGE_MIN=196608" || exit $?
run w2i2d "SVC_MERGE_WAIT_NS=2000000,SVC_INFLIGHT=2,SVC_MERGE_IDLE_NS=100000" || exit $?
run w2i3 "SVC_MERGE_WAIT_NS=2000000,SVC_INFLIGHT=3,SVC_BATCH_MAX=524288,SVC_MERGE_MIN=262144" || exit $?
