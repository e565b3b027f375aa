#!/bin/bash
# round 5 session ai: the paced link (quic_verify depth 16384, no flow control) lost most frags in r05ah's bench;
# the GPU tile's hardware queues (16 vs 4) and the capped gather at the paced configuration
out=gpurun_out/r05ai; mkdir -p $out
export TMPDIR=/tmp
run() { # name svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles 2 --prelay --in-depth 16384 \
    --rate 10000000,5000000 --env "SVC_RUN_REQ_DEPTH=64,SVC_RUN_SLOT_CAP=8192" --svc-env "$2" \
    --logdir $out/logs_$1 >> $out/paced_$1.jsonl 2>> $out/paced.err
}
run a_q16 "" || exit $?
run b_q4 "SVC_HW_QUEUES=4" || exit $?
run c_q16g0 "FD_VERIFY_SVC_GATHER_WGS=0,FD_VERIFY_SVC_FLUSH_WGS=0" || exit $?
run d_q4g0 "SVC_HW_QUEUES=4,FD_VERIFY_SVC_GATHER_WGS=0,FD_VERIFY_SVC_FLUSH_WGS=0" || exit $?
run e_q8 "SVC_HW_QUEUES=8" || exit $?
