#!/bin/bash
# round 5 session u:
#  1. a per-launch timeline of the 2- and 3-tile service runs (kernel trace kept, gzipped)
#  2. the gather's grid capped (FD_VERIFY_SVC_GATHER_WGS) against one wave per frag
#  3. C4 resident (no PCIe kernels beside it) at smaller launch sizes
out=gpurun_out/r05u; mkdir -p $out
export TMPDIR=/tmp
for t in 2 3; do
  timeout -k 10 240 python -u tools/svc_bench.py --frags 4194304 --tiles $t --prelay --env SVC_RUN_REQ_DEPTH=8 \
    --rocprof $out/prof --timeout 200 --logdir $out/logs$t > $out/prof$t.jsonl 2> $out/prof$t.err || exit $?
  f=$(ls $out/prof/t${t}_0/*kernel_trace.csv)
  python3 tools/svc_timeline.py $f > $out/timeline_t$t.json || exit $?
  gzip -c $f > $out/kernel_trace_t$t.csv.gz
  find $out/prof -name "*trace*.csv" -delete
done
run() { # name tiles svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "SVC_RUN_REQ_DEPTH=8" --svc-env "$3" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
run g0 2,3 "FD_VERIFY_SVC_GATHER_WGS=0" || exit $?
run g256 2,3 "FD_VERIFY_SVC_GATHER_WGS=256" || exit $?
run g1024 2,3 "FD_VERIFY_SVC_GATHER_WGS=1024" || exit $?
run g0b 2,3 "FD_VERIFY_SVC_GATHER_WGS=0" || exit $?
for n in 131072 262144; do
  timeout -k 10 200 python -u bench.py --config c4 --txns $n --tiles 1 --steps 20 --warmup 3 --no-tile --no-cpu-baseline \
    > $out/c4t1_$n.json 2> $out/c4t1_$n.err || exit $?
done
for n in 262144 1048576; do
  timeout -k 10 200 python -u bench.py --config c4 --txns $n --steps 20 --warmup 3 --no-tile --no-cpu-baseline \
    > $out/c4_$n.json 2> $out/c4_$n.err || exit $?
done
