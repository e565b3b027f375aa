#!/bin/bash
# round 5 session l: no-memcpy service -- GPU tests, policy sweep, HIP API trace
out=gpurun_out/r05l; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_svc_run.py > $out/pytest.txt 2>&1 || exit $?
run() { # name tiles run-env svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay --env "$3" \
    --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
run base 2,3 "SVC_RUN_REQ_DEPTH=8" "SVC_MERGE_WAIT_NS=400000" || exit $?
run w2i2 2,3,4 "SVC_RUN_REQ_DEPTH=8" "SVC_MERGE_WAIT_NS=2000000,SVC_INFLIGHT=2" || exit $?
run w2i2d16 2,3 "SVC_RUN_REQ_DEPTH=16" "SVC_MERGE_WAIT_NS=2000000,SVC_INFLIGHT=2" || exit $?
run v1 2,3 "SVC_RUN_REQ_DEPTH=16" "SVC_INFLIGHT=2,SVC_MERGE_WAIT_NS=2000000,SVC_MERGE_IDLE_NS=2000000,SVC_MERGE_MIN=262144,SVC_BATCH_MAX=524288" || exit $?
SVC_BENCH_HIP_TRACE=1 timeout -k 10 240 python -u tools/svc_bench.py --frags 4194304 --tiles 3 --prelay --env SVC_RUN_REQ_DEPTH=8 \
  --svc-env SVC_MERGE_WAIT_NS=2000000,SVC_INFLIGHT=2 --rocprof $out/prof --timeout 200 --logdir $out/logsp > $out/prof.jsonl 2> $out/prof.err;
# keep only the summaries: the API trace of a polling loop is hundreds of MiB
find $out/prof -name "*trace*.csv" -delete
du -sh $out
