#!/bin/bash
# round 5 session ao: the GPU tile's DSM reserve default (128) -- service and tile GPU tests, smoke, the default bench line
out=gpurun_out/r05ao; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_svc_run.py tests/test_gpu_tile_run.py > $out/pytest_svc_tile.txt 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || exit $?
