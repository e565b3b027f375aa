#!/bin/bash
# round 5 session x: flush grid capped at 256 by default; where the slots are while the run is active;
# three launches in flight with more outstanding work per tile
out=gpurun_out/r05x; mkdir -p $out
export TMPDIR=/tmp
run() { # name tiles env svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "$3" --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
D8=SVC_RUN_REQ_DEPTH=8; D16=SVC_RUN_REQ_DEPTH=16
run a_def 1,2,3,4 $D8 "" || exit $?
run b_i3d16 2,3 $D16 "SVC_INFLIGHT=3" || exit $?
run c_i3d16w4 2,3 $D16 "SVC_INFLIGHT=3,SVC_MERGE_WAIT_NS=4000000" || exit $?
run d_d16w4 2,3 $D16 "SVC_MERGE_WAIT_NS=4000000" || exit $?
run e_def 2,3 $D8 "" || exit $?
