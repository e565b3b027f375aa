#!/bin/bash
# round 5 session ae: the mirror off by default and its stream created only when on; the box's speed
# (host CPU, a short C4 leg) beside the service A/B
out=gpurun_out/r05ae; mkdir -p $out
export TMPDIR=/tmp
lscpu | grep "Model name" > $out/host.txt
run() { # name tiles env svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "$3" --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
D8=SVC_RUN_REQ_DEPTH=8
run a_def 2,3 $D8 "" || exit $?
run b_m1 2,3 $D8 "FD_VERIFY_SVC_MIRROR=1" || exit $?
run c_def 2,3 $D8 "" || exit $?
timeout -k 10 200 python -u bench.py --config c4 --steps 10 --warmup 2 --no-tile --no-cpu-baseline > $out/c4.json 2> $out/c4.err || exit $?
