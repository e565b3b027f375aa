#!/bin/bash
# round 5 session t: flushes through the copy engine (HBM mirror + DMA) vs the flush kernel writing host memory
out=gpurun_out/r05t; mkdir -p $out
export TMPDIR=/tmp
FD_VERIFY_SVC_FLUSH_DMA=1 timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_svc_run.py > $out/pytest_dma.txt 2>&1 || exit $?
run() { # name tiles svc-env
  timeout -k 10 150 python -u tools/svc_bench.py --frags 4194304 --tiles $2 --repeat 2 --prelay \
    --env "SVC_RUN_REQ_DEPTH=8" --svc-env "$3" --logdir $out/logs_$1 >> $out/bench_$1.jsonl 2>> $out/bench.err
}
run k1 2,3 "FD_VERIFY_SVC_FLUSH_DMA=0" || exit $?
run d1 2,3 "FD_VERIFY_SVC_FLUSH_DMA=1" || exit $?
run k2 2,3 "FD_VERIFY_SVC_FLUSH_DMA=0" || exit $?
run d2 2,3 "FD_VERIFY_SVC_FLUSH_DMA=1" || exit $?
timeout -k 10 240 python -u tools/svc_bench.py --frags 4194304 --tiles 2 --prelay --env SVC_RUN_REQ_DEPTH=8 \
  --svc-env FD_VERIFY_SVC_FLUSH_DMA=1 --rocprof $out/prof --timeout 200 --logdir $out/logsp > $out/prof.jsonl 2> $out/prof.err || exit $?
python3 tools/trace_util.py $out/prof/t2_0 > $out/util_t2_dma.json
find $out/prof -name "*trace*.csv" -delete
