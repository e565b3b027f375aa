#!/bin/bash
# round 5 session n: hardware queues for the GPU tile (ingest / flush streams not behind verify launches)
out=gpurun_out/r05n; mkdir -p $out
export TMPDIR=/tmp
run() { # name tiles run-env svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay --env "$3" \
    --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
run q4 2,3 "SVC_RUN_REQ_DEPTH=8" "GPU_MAX_HW_QUEUES=4" || exit $?
run q16 2,3,4 "SVC_RUN_REQ_DEPTH=8" "GPU_MAX_HW_QUEUES=16" || exit $?
run q16i3 2,3 "SVC_RUN_REQ_DEPTH=8" "GPU_MAX_HW_QUEUES=16,SVC_INFLIGHT=3" || exit $?
timeout -k 10 400 python -u tools/svc_link_sweep.py --frags 4194304 --tiles 2 --steps 4 --depths 16384,65536,262144 \
  --env SVC_RUN_REQ_DEPTH=64,SVC_RUN_SLOT_CAP=8192 --svc-env GPU_MAX_HW_QUEUES=16 --logdir $out/logsw > $out/sweep.jsonl 2> $out/sweep.err
