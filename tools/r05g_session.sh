#!/bin/bash
# round 5 session g: the direct patch's stalled-consumer tests, the service GPU tests, then the pinned sweep
out=gpurun_out/r05g; mkdir -p $out
for d in /sys/bus/pci/devices/*; do v=$(cat $d/vendor); c=$(cat $d/class); if [ "$v" = "0x1002" ]; then echo "$d $c $(cat $d/numa_node)"; fi; done > $out/gpu_numa.txt
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fec.py tests/test_gpu_tile_run.py -k "stalled or fec" > $out/pytest.txt 2>&1 && timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_svc_run.py >> $out/pytest.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/svc_bench.py --frags 4194304 --tiles 2,3,4 --repeat 2 --prelay --env SVC_RUN_REQ_DEPTH=8 --logdir $out/logs > $out/bench.jsonl 2> $out/bench.err || exit $?
timeout -k 10 200 python -u tools/svc_bench.py --frags 4194304 --tiles 2,3 --prelay --pin none --env SVC_RUN_REQ_DEPTH=8 --logdir $out/logsn >> $out/bench.jsonl 2>> $out/bench.err
