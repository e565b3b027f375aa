#!/bin/bash
# round 5 session ag: the GPU tile now sets GPU_MAX_HW_QUEUES=16 over the box's exported 4 -- A/B with 4,
# and the mirror again at 16 queues
out=gpurun_out/r05ag; mkdir -p $out
export TMPDIR=/tmp
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset}" > $out/host.txt
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_svc_run.py > $out/pytest_svc.txt 2>&1 || exit $?
run() { # name tiles env svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "$3" --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
D8=SVC_RUN_REQ_DEPTH=8
run a_q16 2,3 $D8 "" || exit $?
run b_q4 2,3 $D8 "SVC_HW_QUEUES=4" || exit $?
run c_q16m1 2,3 $D8 "FD_VERIFY_SVC_MIRROR=1" || exit $?
run d_q16 2,3 $D8 "" || exit $?
run e_q16m1 2,3 $D8 "FD_VERIFY_SVC_MIRROR=1" || exit $?
run f_q16d16 2,3 SVC_RUN_REQ_DEPTH=16 "" || exit $?
run g_q16i3 2,3 $D8 "SVC_INFLIGHT=3" || exit $?
