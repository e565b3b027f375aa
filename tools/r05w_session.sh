#!/bin/bash
# round 5 session w: the gather capped at 256 workgroups by default -- the service tests, where the slots
# are (occupancy), and the flush kernel's cap / gather caps around 256
out=gpurun_out/r05w; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_svc_run.py > $out/pytest_svc.txt 2>&1 || exit $?
run() { # name tiles env svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "$3" --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
D8=SVC_RUN_REQ_DEPTH=8; D16=SVC_RUN_REQ_DEPTH=16
run a_def 2,3 $D8 "" || exit $?
run b_f128 2,3 $D8 "FD_VERIFY_SVC_FLUSH_WGS=128" || exit $?
run c_f256 2,3 $D8 "FD_VERIFY_SVC_FLUSH_WGS=256" || exit $?
run d_f512 2,3 $D8 "FD_VERIFY_SVC_FLUSH_WGS=512" || exit $?
run e_g384 2,3 $D8 "FD_VERIFY_SVC_GATHER_WGS=384" || exit $?
run f_g512 2,3 $D8 "FD_VERIFY_SVC_GATHER_WGS=512" || exit $?
run g_d16 2,3 $D16 "" || exit $?
run h_def 2,3 $D8 "" || exit $?
