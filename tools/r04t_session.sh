#!/bin/bash
set -o pipefail
O=gpurun_out/r04t; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tile_run.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
