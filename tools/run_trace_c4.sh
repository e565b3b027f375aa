#!/bin/bash
# GPU-box script: rocprofv3 kernel + memory-copy trace of the default C4 bench
# (tools/trace_busy.py reads the timed resident steps out of it).
# Usage: bash tools/run_trace_c4.sh <tag> [bench args...]
export TMPDIR=/tmp
T=${1:-c4trace}; shift
O=$PWD/gpurun_out/$T; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o run -- \
    python3 bench.py --config c4 --no-cpu-baseline --steps 6 --warmup 2 "$@" > $O/bench.json 2> $O/bench.err
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
f=$(find $O/tr -name '*kernel_trace.csv' | head -1)
python3 tools/trace_busy.py $f 6 2 6 > $O/busy.json && cat $O/busy.json
