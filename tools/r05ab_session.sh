#!/bin/bash
# round 5 session ab: range frags reach HBM by DMA of the link's data region (the link mirror) --
# the service tests with it on, then an A/B against the gather reading each frag over PCIe
out=gpurun_out/r05ab; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_svc_run.py > $out/pytest_svc.txt 2>&1 || exit $?
run() { # name tiles env svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "$3" --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
D8=SVC_RUN_REQ_DEPTH=8
run a_m1 2,3 $D8 "FD_VERIFY_SVC_MIRROR=1" || exit $?
run b_m0 2,3 $D8 "FD_VERIFY_SVC_MIRROR=0" || exit $?
run c_m1 2,3 $D8 "FD_VERIFY_SVC_MIRROR=1" || exit $?
run d_m0 2,3 $D8 "FD_VERIFY_SVC_MIRROR=0" || exit $?
run e_m1d16 2,3 SVC_RUN_REQ_DEPTH=16 "FD_VERIFY_SVC_MIRROR=1" || exit $?
run f_m1o64k 2,3 "$D8,SVC_RUN_OUT_DEPTH=65536" "FD_VERIFY_SVC_MIRROR=1" || exit $?
timeout -k 10 240 python -u tools/svc_bench.py --frags 4194304 --tiles 2 --prelay --env $D8 \
  --rocprof $out/prof --timeout 200 --logdir $out/logsp > $out/prof.jsonl 2> $out/prof.err || exit $?
f=$(ls $out/prof/t2_0/*kernel_trace.csv)
python3 tools/svc_timeline.py $f > $out/timeline_t2.json || exit $?
python3 tools/trace_util.py $out/prof/t2_0 > $out/util_t2.json
gzip -c $f > $out/kernel_trace_t2.csv.gz
find $out/prof -name "*trace*.csv" -delete
