#!/bin/bash
# round 5 session al: the tile's overrun check at INGESTED finds the reused prefix of a range once (bisection)
# instead of re-reading each frag's line at the ordered pass, which also dropped frags reused after the GPU's
# read -- the service tests, then the link-conditions sweep
out=gpurun_out/r05al; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_svc_run.py > $out/pytest_svc.txt 2>&1 || exit $?
timeout -k 10 500 python -u tools/svc_link_sweep.py --frags 4194304 --tiles 2 --steps 4 --depths 16384,65536,262144 \
  --env SVC_RUN_REQ_DEPTH=64,SVC_RUN_SLOT_CAP=8192 --logdir $out/logsw2 > $out/sweep_t2.jsonl 2> $out/sweep_t2.err || exit $?
timeout -k 10 500 python -u tools/svc_link_sweep.py --frags 4194304 --tiles 3 --steps 4 --depths 16384 \
  --env SVC_RUN_REQ_DEPTH=64,SVC_RUN_SLOT_CAP=8192 --logdir $out/logsw3 > $out/sweep_t3.jsonl 2> $out/sweep_t3.err || exit $?
