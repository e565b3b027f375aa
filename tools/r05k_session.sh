#!/bin/bash
# round 5 session k: large verify launches (merge policy without the idle trigger), link sweep with more,
# smaller request slots, the replay block path through the scheduler
out=gpurun_out/r05k; mkdir -p $out
export TMPDIR=/tmp
run() { # name tiles run-env svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay --env "$3" \
    --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
run v1 2,3 "SVC_RUN_REQ_DEPTH=16" "SVC_INFLIGHT=2,SVC_MERGE_WAIT_NS=2000000,SVC_MERGE_IDLE_NS=2000000,SVC_MERGE_MIN=262144,SVC_BATCH_MAX=524288" || exit $?
run v2 2,3 "SVC_RUN_REQ_DEPTH=16" "SVC_INFLIGHT=2,SVC_MERGE_WAIT_NS=1000000,SVC_MERGE_IDLE_NS=1000000,SVC_MERGE_MIN=196608,SVC_BATCH_MAX=393216" || exit $?
run v3 2,3 "SVC_RUN_REQ_DEPTH=16" "SVC_INFLIGHT=1,SVC_MERGE_WAIT_NS=2000000,SVC_MERGE_IDLE_NS=2000000,SVC_MERGE_MIN=262144,SVC_BATCH_MAX=524288" || exit $?
run v1t4 4 "SVC_RUN_REQ_DEPTH=8" "SVC_INFLIGHT=2,SVC_MERGE_WAIT_NS=2000000,SVC_MERGE_IDLE_NS=2000000,SVC_MERGE_MIN=262144,SVC_BATCH_MAX=524288" || exit $?
timeout -k 10 400 python -u tools/svc_link_sweep.py --frags 4194304 --tiles 2 --steps 4 --depths 16384,65536 \
  --env SVC_RUN_REQ_DEPTH=64,SVC_RUN_SLOT_CAP=8192 --logdir $out/logsw > $out/sweep.jsonl 2> $out/sweep.err || exit $?
timeout -k 10 400 python -u tools/replay_block_bench.py --txns 16384,98039 --reps 10 --sched > $out/replay.jsonl 2> $out/replay.err
