#!/bin/bash
# round 5 session y: the DSM grid leaves some workgroup slots free (FD_ED25519_HIP_DSM_RESERVE) so that the
# gather and flush kernels are not held back for a whole DSM pass
out=gpurun_out/r05y; mkdir -p $out
export TMPDIR=/tmp
run() { # name tiles env svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "$3" --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
D8=SVC_RUN_REQ_DEPTH=8
run a_def 2,3 $D8 "" || exit $?
run b_r64 2,3 $D8 "FD_ED25519_HIP_DSM_RESERVE=64" || exit $?
run c_r128 2,3 $D8 "FD_ED25519_HIP_DSM_RESERVE=128" || exit $?
run d_r256 2,3 $D8 "FD_ED25519_HIP_DSM_RESERVE=256" || exit $?
run e_def 2,3 $D8 "" || exit $?
run f_r128 2,3 $D8 "FD_ED25519_HIP_DSM_RESERVE=128" || exit $?
