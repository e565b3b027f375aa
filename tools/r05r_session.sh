#!/bin/bash
# round 5 session r: 16 lanes per frag in the PCIe kernels (A/B), with the GPU tile on 3 cores
out=gpurun_out/r05r; mkdir -p $out
export TMPDIR=/tmp
run() { # name tiles run-env svc-env
  SVC_BENCH_SVC_CORES=3 timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "$3" --svc-env "$4" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
run l64 2,3 "SVC_RUN_REQ_DEPTH=8" "FD_VERIFY_SVC_LPF=64" || exit $?
run l16 2,3 "SVC_RUN_REQ_DEPTH=8" "FD_VERIFY_SVC_LPF=16" || exit $?
run l64b 2,3 "SVC_RUN_REQ_DEPTH=8" "FD_VERIFY_SVC_LPF=64" || exit $?
run l16b 2,3 "SVC_RUN_REQ_DEPTH=8" "FD_VERIFY_SVC_LPF=16" || exit $?
FD_VERIFY_SVC_LPF=16 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_svc_run.py -k "one_tile or two_tiles or scale" > $out/pytest_l16.txt 2>&1
