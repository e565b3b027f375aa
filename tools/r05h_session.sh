#!/bin/bash
# round 5 session h: a kernel/copy trace of the GPU tile under load, the link-conditions sweep, the default bench line
out=gpurun_out/r05h; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/svc_bench.py --frags 4194304 --tiles 2 --prelay --env SVC_RUN_REQ_DEPTH=8 --rocprof $out/prof --timeout 200 --logdir $out/logsp > $out/prof.jsonl 2> $out/prof.err || exit $?
timeout -k 10 500 python -u tools/svc_link_sweep.py --frags 4194304 --tiles 2 --steps 4 --logdir $out/logsw > $out/sweep.jsonl 2> $out/sweep.err || exit $?
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err
