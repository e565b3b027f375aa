#!/bin/bash
# GPU-box script: the VALU issue-slot PMC pass of tools/run_valu_calib.sh over
# the C4 verify-tile bench instead of the C2 batch, so that C4's roofline is
# read from C4's own k_verify_dsm dispatch (the last one of the run: the
# timing leg's tile-0 batch) and not scaled from C2's.  One pass, no trace
# domains besides --kernel-trace.
# Usage: bash tools/run_c4_issue.sh <tag>  -> gpurun_out/c4issue_<tag>/
export TMPDIR=/tmp
R=$(pwd); T=${1:-r03}; O=$R/gpurun_out/c4issue_$T; mkdir -p $O
G="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 300 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/engine -o run -- \
    python3 bench.py --config c4 --no-cpu-baseline --steps 2 --warmup 1 --c4-pcie-steps 1 > $O/bench.json 2> $O/engine.err
rc=$?; echo "c4 pmc rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/engine.err; exit $rc; }
exit 0
