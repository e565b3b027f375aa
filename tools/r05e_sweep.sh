#!/bin/bash
out=gpurun_out/r05e; mkdir -p $out
timeout -k 10 300 python -u tools/svc_bench.py --frags 4194304 --tiles 2,3 --repeat 2 --prelay --logdir $out/logs > $out/bench.jsonl 2> $out/bench.err || exit $?
timeout -k 10 200 python -u tools/svc_bench.py --frags 4194304 --tiles 4 --prelay --env SVC_RUN_REQ_DEPTH=8 --logdir $out/logs4 >> $out/bench.jsonl 2>> $out/bench.err || exit $?
timeout -k 10 200 python -u tools/svc_bench.py --frags 4194304 --tiles 2,3 --prelay --svc-env SVC_MERGE_MIN=200000,SVC_MERGE_WAIT_NS=1000000 --logdir $out/logsm >> $out/bench.jsonl 2>> $out/bench.err
