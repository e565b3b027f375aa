#!/bin/bash
# GPU-box script: kernel-trace statistics of the bench command, then rocprofv3
# PMC passes (one counter group per run, no trace domains mixed in).  Runs
# bench.py --contexts 1, so that every k_verify_dsm dispatch is a whole
# 2^20-signature batch: the rocprof per-dispatch averages then describe the
# same launch as bench.py's roofline leg (its traffic and duration).
# Usage: bash tools/run_profile.sh <tag>   -> gpurun_out/prof_<tag>/...
export TMPDIR=/tmp
R=$(pwd)
T=${1:-r01}
O=$R/gpurun_out/prof_$T
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --contexts 1 --no-c4 --no-tile > $O/bench_stats.json 2> $O/bench_stats.err
rc=$?; echo "stats rc=$rc"
if [ $rc -ne 0 ]; then tail -20 $O/bench_stats.err; exit $rc; fi
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" ; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -o run -- \
      python3 bench.py --contexts 1 --no-c4 --no-tile --no-cpu-baseline --steps 2 --warmup 1 > $O/p$i.out 2> $O/p$i.err
  rc=$?
  echo "pass $i [$grp] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/p$i.err; exit $rc; fi
done
exit 0
