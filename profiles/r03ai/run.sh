#!/bin/bash
# r03ai: where C4's prep time goes -- one rocprofv3 PMC pass (8 SQ + 2 GRBM
# counters, no trace domains) over C4 with one tile taking all 2^20 frags
# (9 rounds of resident waves: no launch tail) and over C2 (contexts 1)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r03ai; mkdir -p $O
G="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 300 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/c4 -o run -- \
    python3 bench.py --config c4 --no-cpu-baseline --steps 1 --warmup 1 --tiles 1 --c4-pcie-steps 1 > $O/c4.out 2> $O/c4.err
rc=$?; echo "c4 pass rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/c4.err; exit $rc; }
timeout -s KILL 300 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/c2 -o run -- \
    python3 bench.py --contexts 1 --no-cpu-baseline --steps 2 --warmup 1 > $O/c2.out 2> $O/c2.err
rc=$?; echo "c2 pass rc=$rc"; exit $rc
