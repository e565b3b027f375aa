#!/bin/bash
# GPU-box script: one rocprofv3 PMC pass (8 SQ + 2 GRBM counters, no trace
# domains; PMC collection serialises dispatches, so per-dispatch values are
# clean) over the C4 bench, for k_verify_prep's issue-slot use and waits.
export TMPDIR=/tmp
R=$(pwd); T=${1:-r02}; O=$R/gpurun_out/c4prep_$T; mkdir -p $O
G="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 300 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/p -o run -- \
    python3 bench.py --config c4 --no-cpu-baseline --steps 2 --warmup 1 --tiles 2 --txns 524288 > $O/p.out 2> $O/p.err
rc=$?; echo "c4 pass rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/p.err; exit $rc; }
timeout -s KILL 300 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/c2 -o run -- \
    python3 bench.py --contexts 1 --no-cpu-baseline --steps 2 --warmup 1 > $O/c2.out 2> $O/c2.err
rc=$?; echo "c2 pass rc=$rc"; exit $rc
