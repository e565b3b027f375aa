#!/bin/bash
# round 5 session p: kernel-class timelines of the service under load (T2, T3)
out=gpurun_out/r05p; mkdir -p $out
export TMPDIR=/tmp
for t in 2 3; do
  timeout -k 10 240 python -u tools/svc_bench.py --frags 4194304 --tiles $t --prelay --env SVC_RUN_REQ_DEPTH=8 \
    --rocprof $out/prof --timeout 200 --logdir $out/logs$t >> $out/prof.jsonl 2>> $out/prof.err || exit $?
  python3 tools/trace_util.py $out/prof/t${t}_0 > $out/util_t$t.json
  find $out/prof/t${t}_0 -name "*trace*.csv" -delete
done
