#!/bin/bash
# r03z: single-call drop-in latency on HEAD (tools/bench_latency.py, 500 calls per entry point)
set -o pipefail
O=gpurun_out/r03z; mkdir -p $O
timeout -k 10 300 python3 tools/bench_latency.py 500 > $O/dropin_latency.json 2> $O/err.txt || { tail -10 $O/err.txt; exit 1; }
cat $O/dropin_latency.json
