#!/bin/bash
# r03d: full GPU suite on the concurrent drop-in slots, drop-in slot-count A/B (C callers), C2 bench
set -o pipefail
O=gpurun_out/r03d; mkdir -p $O
export FD_DROPIN_SUMMARY=$O/dropin_slots4.json
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -3 $O/pytest_gpu.txt
for k in 1 2 8; do
  FD_ED25519_HIP_DROPIN_SLOTS=$k FD_DROPIN_SUMMARY=$O/dropin_slots$k.json timeout -k 10 150 \
    python -u -m pytest tests/test_gpu_dropin_concurrent.py -k c_callers -s --timeout 140 --timeout-method thread > $O/dropin_slots$k.txt 2>&1 || { tail -20 $O/dropin_slots$k.txt; exit 1; }
  grep "C callers" $O/dropin_slots$k.txt
done
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json | cut -c1-400
bash tools/run_ab.sh micro "" $PWD/firedancer_amd/libfd_ed25519_hip_base.so
