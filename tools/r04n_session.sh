mkdir -p gpurun_out/r04n
timeout -k 10 700 python -u -m pytest tests/test_gpu_replay_block.py tests/test_gpu_replay.py tests/test_gpu_txn_batch.py tests/test_gpu_tile_hip.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r04n/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r04n/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/replay_block_bench.py --txns 16384,98039 --sched > gpurun_out/r04n/replay_bench.jsonl 2> gpurun_out/r04n/replay_bench.err
rc=$?; cat gpurun_out/r04n/replay_bench.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tile_bench.py --frags 2097152 --tiles 1,2,4 --configs b4096i4,b8192i4,b2048i2 --timeout 90 --logdir gpurun_out/r04n/logs > gpurun_out/r04n/sweep.jsonl 2> gpurun_out/r04n/sweep.err
rc=$?; tail -2 gpurun_out/r04n/sweep.jsonl; exit $rc
