#!/bin/bash
# round 5 session an: the DSM grid reserve (128 workgroup slots) in the GPU tile's contexts, A/B x3 on the final service
out=gpurun_out/r05an; mkdir -p $out
export TMPDIR=/tmp
run() { # name tiles env svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "$3" --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
D8=SVC_RUN_REQ_DEPTH=8
for k in 1 2 3; do
  run r0_$k 2,3 $D8 "" || exit $?
  run r128_$k 2,3 $D8 "FD_ED25519_HIP_DSM_RESERVE=128" || exit $?
done
