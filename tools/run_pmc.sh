#!/bin/bash
# GPU-box script: rocprofv3 PMC passes (one counter group per run, no trace domains mixed in).
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || rocprofv3 --list-avail > gpurun_out/pmc/counters_list.txt 2>&1
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" \
           "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- \
      python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/pmc/p$i.out 2> gpurun_out/pmc/p$i.err
  rc=$?
  echo "pass $i [$grp] rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
exit 0
