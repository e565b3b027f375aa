#!/bin/bash
# round 5 session ad: the link mirror A/B on a third box
out=gpurun_out/r05ad; mkdir -p $out
export TMPDIR=/tmp
nproc > $out/host.txt; lscpu | head -20 >> $out/host.txt
run() { # name tiles env svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "$3" --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
D8=SVC_RUN_REQ_DEPTH=8
run a_m0 2,3 $D8 "FD_VERIFY_SVC_MIRROR=0" || exit $?
run b_m1 2,3 $D8 "FD_VERIFY_SVC_MIRROR=1" || exit $?
run c_m0 2,3 $D8 "FD_VERIFY_SVC_MIRROR=0" || exit $?
run d_m1 2,3 $D8 "FD_VERIFY_SVC_MIRROR=1" || exit $?
