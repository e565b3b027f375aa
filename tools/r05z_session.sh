#!/bin/bash
# round 5 session z: is the out link's credit loop the bound? a deeper verify_dedup link (SVC_RUN_OUT_DEPTH),
# smaller flushes (FD_VERIFY_SVC_FLUSH_MIN 1024 / 2048: build variants of the tile driver), DSM reserve 128
out=gpurun_out/r05z; mkdir -p $out
export TMPDIR=/tmp
run() { # name tiles env svc-env [exe]
  SVC_BENCH_TILE_EXE=${5:-integration/_build/svc_tile_run} timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 \
    --tiles $2 --repeat 2 --prelay --env "$3" --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
D8=SVC_RUN_REQ_DEPTH=8
run a_def 2,3 $D8 "" || exit $?
run b_o64k 2,3 "$D8,SVC_RUN_OUT_DEPTH=65536" "" || exit $?
run c_fm1024 2,3 $D8 "" integration/_build/svc_tile_run_fm1024 || exit $?
run d_fm2048 2,3 $D8 "" integration/_build/svc_tile_run_fm2048 || exit $?
run e_fm1024r128 2,3 $D8 "FD_ED25519_HIP_DSM_RESERVE=128" integration/_build/svc_tile_run_fm1024 || exit $?
run f_o64kd16 2,3 "SVC_RUN_REQ_DEPTH=16,SVC_RUN_OUT_DEPTH=65536" "" || exit $?
