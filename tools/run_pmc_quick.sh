#!/bin/bash
# GPU-box script: one rocprofv3 PMC pass (counters given as arguments) over a short bench.
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/pmcq
timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $R/gpurun_out/pmcq -o run -- \
    python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/pmcq/out.txt 2> gpurun_out/pmcq/err.txt
rc=$?; echo "rc=$rc"; exit $rc
