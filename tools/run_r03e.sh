#!/bin/bash
# r03e: is the lone latency-kernel workgroup instruction-fetch bound?
#  (1) icache/ifetch PMC pass over 1-thread drop-in calls (C harness, one slot: 8 racing copies)
#  (2) C-caller latency A/B: default vs FD_LAT_IPREF=1 (idle waves pull the kernel's code into L2)
#  (3) the micro A/B that failed in r03d (default vs base build on C2)
set -o pipefail
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03e; mkdir -p $O
timeout -k 10 120 python3 -c "import sys; sys.path.insert(0,'tests'); from test_gpu_dropin_concurrent import _harness_input; _harness_input('$O/calls.bin', 64, 12, 64, 0x1612)" || exit 1
G="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"
FD_ED25519_HIP_DROPIN_SLOTS=1 timeout -s KILL 90 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/pmc -o run -- \
    $R/tools/dropin_threads $O/calls.bin 1 1 > $O/pmc_out.json 2> $O/pmc_err.txt
echo "pmc rc=$?"
mkdir -p $O/v_ipref && ln -sf $R/firedancer_amd/libfd_ed25519_hip_ipref.so $O/v_ipref/libfd_ed25519_hip.so
for rep in 1 2; do
  for v in default ipref; do
    for sl in 1 4; do
      LP=""; [ $v = ipref ] && LP=$O/v_ipref
      for th in 1 16; do
        LD_LIBRARY_PATH=$LP FD_ED25519_HIP_DROPIN_SLOTS=$sl timeout -k 10 60 $R/tools/dropin_threads $O/calls.bin 2 $th > $O/h_${v}_s${sl}_t${th}_$rep.json 2>> $O/h_err.txt || { echo "harness $v $sl $th failed"; tail -5 $O/h_err.txt; exit 1; }
        python3 -c "import json; d=json.load(open('$O/h_${v}_s${sl}_t${th}_$rep.json')); print('$v slots $sl threads $th rep $rep', round(d['sigs_per_s']/1e6,3), 'M/s p50', d['p50_us'], 'p99', d['p99_us'], 'cpl', d['calls_per_launch'])"
      done
    done
  done
done
sed -i 's#pytest_${v:-default}#pytest_$(basename ${v:-default})#g; s#bench_${v:-default}#bench_$(basename ${v:-default})#g' tools/run_ab.sh
bash tools/run_ab.sh micro "" $R/firedancer_amd/libfd_ed25519_hip_base.so
