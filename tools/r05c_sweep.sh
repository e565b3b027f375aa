#!/bin/bash
out=gpurun_out/r05c; mkdir -p $out
for cfg in "2:" "1:" "3:" "4:" "2:SVC_BATCH_MAX=262144" "2:SVC_INFLIGHT=2"; do
  t=${cfg%%:*}; e=${cfg#*:}
  timeout -k 10 200 python -u tools/svc_bench.py --frags 2097152 --tiles $t --prelay --svc-env "$e" --logdir $out/logs_${t}_${e} >> $out/bench.jsonl 2>> $out/bench.err || exit $?
done
