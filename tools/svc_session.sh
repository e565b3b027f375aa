#!/bin/bash
# GPU-box session for the service-mode stage: tests, then a bench sweep.
# usage: tools/svc_session.sh <outdir> [frags] [tiles]
# A test failure (pytest rc 1) still runs the bench; a timeout, abort or
# crash ends the session there.
out=$1; frags=${2:-2097152}; tiles=${3:-1,2,3}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_svc_run.py -x -v --timeout 400 --timeout-method thread > "$out/pytest.txt" 2>&1
rc=$?
echo "pytest rc $rc" >> "$out/pytest.txt"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/svc_bench.py --frags "$frags" --tiles "$tiles" --prelay --logdir "$out/logs" > "$out/bench.jsonl" 2> "$out/bench.err"
exit $?
