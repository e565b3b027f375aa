#!/bin/bash
# round 5 session aq: the DSM reserve at 128 (default) vs 192 / 256 on the final service
out=gpurun_out/r05aq; mkdir -p $out
export TMPDIR=/tmp
run() { # name tiles env svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "$3" --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
D8=SVC_RUN_REQ_DEPTH=8
for k in 1 2; do
  run r128_$k 2,3 $D8 "" || exit $?
  run r192_$k 2,3 $D8 "FD_ED25519_HIP_DSM_RESERVE=192" || exit $?
  run r256_$k 2,3 $D8 "FD_ED25519_HIP_DSM_RESERVE=256" || exit $?
done
