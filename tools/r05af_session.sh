#!/bin/bash
# round 5 session af: the link mirror with its copies on the ingest stream (no extra stream), A/B;
# the service tests with it on
out=gpurun_out/r05af; mkdir -p $out
export TMPDIR=/tmp
lscpu | grep "Model name" > $out/host.txt; echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset}" >> $out/host.txt
FD_VERIFY_SVC_MIRROR=1 timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_svc_run.py > $out/pytest_m1.txt 2>&1 || exit $?
run() { # name tiles env svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "$3" --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
D8=SVC_RUN_REQ_DEPTH=8
run a_m0 2,3 $D8 "" || exit $?
run b_m1 2,3 $D8 "FD_VERIFY_SVC_MIRROR=1" || exit $?
run c_m0 2,3 $D8 "" || exit $?
run d_m1 2,3 $D8 "FD_VERIFY_SVC_MIRROR=1" || exit $?
run e_m1o64k 2,3 "$D8,SVC_RUN_OUT_DEPTH=65536" "FD_VERIFY_SVC_MIRROR=1" || exit $?
