#!/bin/bash
# round 5 session v: the PCIe kernels' grid caps (gather, flush) and more launches in flight
out=gpurun_out/r05v; mkdir -p $out
export TMPDIR=/tmp
run() { # name tiles env svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "$3" --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
D8=SVC_RUN_REQ_DEPTH=8; D16=SVC_RUN_REQ_DEPTH=16
run a_g256 2,3 $D8 "FD_VERIFY_SVC_GATHER_WGS=256" || exit $?
run b_g128 2,3 $D8 "FD_VERIFY_SVC_GATHER_WGS=128" || exit $?
run c_g64 2,3 $D8 "FD_VERIFY_SVC_GATHER_WGS=64" || exit $?
run d_g256f256 2,3 $D8 "FD_VERIFY_SVC_GATHER_WGS=256,FD_VERIFY_SVC_FLUSH_WGS=256" || exit $?
run e_g256f64 2,3 $D8 "FD_VERIFY_SVC_GATHER_WGS=256,FD_VERIFY_SVC_FLUSH_WGS=64" || exit $?
run f_g256i3 2,3 $D8 "FD_VERIFY_SVC_GATHER_WGS=256,SVC_INFLIGHT=3" || exit $?
run g_g256i4m64d16 2,3 $D16 "FD_VERIFY_SVC_GATHER_WGS=256,SVC_INFLIGHT=4,SVC_MERGE_MIN=65536" || exit $?
run h_g256i4b128d16 2,3 $D16 "FD_VERIFY_SVC_GATHER_WGS=256,SVC_INFLIGHT=4,SVC_MERGE_MIN=65536,SVC_BATCH_MAX=131072" || exit $?
run i_g256 2,3 $D8 "FD_VERIFY_SVC_GATHER_WGS=256" || exit $?
