#!/bin/bash
# GPU-box script: hardware VALU issue accounting, calibrated.  One rocprofv3
# PMC pass (8 SQ + 2 GRBM counters, no trace domains) over
#   (1) tools/valu_rates2: one kernel per instruction class, known mix
#   (2) bench.py --contexts 1: the engine's k_verify_prep / k_verify_dsm
# so that SQ_THREAD_CYCLES_VALU per instruction (the hardware's own issue
# cost) and GRBM cycles can be read for known classes and for the engine.
# Usage: bash tools/run_valu_calib.sh <tag>  -> gpurun_out/valu_<tag>/
export TMPDIR=/tmp
R=$(pwd); T=${1:-r02}; O=$R/gpurun_out/valu_$T; mkdir -p $O
G="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 120 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/micro -o run -- \
    $R/tools/valu_rates2 > $O/micro.out 2> $O/micro.err
rc=$?; echo "micro rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/micro.err; exit $rc; }
timeout -s KILL 240 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/engine -o run -- \
    python3 bench.py --contexts 1 --no-c4 --no-tile --no-cpu-baseline --steps 2 --warmup 1 > $O/engine.out 2> $O/engine.err
rc=$?; echo "engine rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/engine.err; exit $rc; }
exit 0
