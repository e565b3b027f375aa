#!/bin/bash
# round 5 session ap: the full GPU suite on the round's final HEAD
out=gpurun_out/r05ap; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || exit $?
