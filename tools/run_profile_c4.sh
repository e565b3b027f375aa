#!/bin/bash
# GPU-box script: rocprofv3 kernel-trace stats + PMC passes (one counter
# group per run, no trace domains mixed in) of the C4 verify-tile bench.
# Usage: bash tools/run_profile_c4.sh <tag>  -> gpurun_out/prof_c4_<tag>/...
export TMPDIR=/tmp
R=$(pwd); T=${1:-r02}; O=$R/gpurun_out/prof_c4_$T; mkdir -p $O
ARGS="--config c4 --no-cpu-baseline --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py $ARGS > $O/bench_stats.json 2> $O/bench_stats.err
rc=$?; echo "stats rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench_stats.err; exit $rc; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -o run -- \
      python3 bench.py $ARGS > $O/p$i.out 2> $O/p$i.err
  rc=$?; echo "pass $i [$grp] rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $O/p$i.err; exit $rc; }
done
exit 0
