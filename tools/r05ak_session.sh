#!/bin/bash
# round 5 session ak: the link-conditions sweep again on the round's final service (capped PCIe kernels,
# 8 hardware queues in the GPU tile), 2 and 3 tiles
out=gpurun_out/r05ak; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/svc_link_sweep.py --frags 4194304 --tiles 2 --steps 4 --depths 16384,65536,262144 \
  --env SVC_RUN_REQ_DEPTH=64,SVC_RUN_SLOT_CAP=8192 --logdir $out/logsw2 > $out/sweep_t2.jsonl 2> $out/sweep_t2.err || exit $?
timeout -k 10 500 python -u tools/svc_link_sweep.py --frags 4194304 --tiles 3 --steps 4 --depths 16384 \
  --env SVC_RUN_REQ_DEPTH=64,SVC_RUN_SLOT_CAP=8192 --logdir $out/logsw3 > $out/sweep_t3.jsonl 2> $out/sweep_t3.err || exit $?
