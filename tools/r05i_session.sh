#!/bin/bash
# round 5 session i: early ingest (INGESTED state) -- service GPU tests, tile sweep, merge variants, link sweep
out=gpurun_out/r05i; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_svc_run.py > $out/pytest.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/svc_bench.py --frags 4194304 --tiles 1,2,3,4 --repeat 2 --prelay --env SVC_RUN_REQ_DEPTH=8 --logdir $out/logs > $out/bench.jsonl 2> $out/bench.err || exit $?
timeout -k 10 200 python -u tools/svc_bench.py --frags 4194304 --tiles 2,3 --repeat 2 --prelay --env SVC_RUN_REQ_DEPTH=8 --svc-env SVC_MERGE_IDLE_NS=150000 --logdir $out/logsm > $out/bench_m.jsonl 2> $out/bench_m.err || exit $?
timeout -k 10 240 python -u tools/svc_bench.py --frags 4194304 --tiles 2 --prelay --env SVC_RUN_REQ_DEPTH=8 --rocprof $out/prof --timeout 200 --logdir $out/logsp > $out/prof.jsonl 2> $out/prof.err || exit $?
timeout -k 10 400 python -u tools/svc_link_sweep.py --frags 4194304 --tiles 2 --steps 4 --depths 16384,65536 --logdir $out/logsw > $out/sweep.jsonl 2> $out/sweep.err
