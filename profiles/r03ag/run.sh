#!/bin/bash
# r03ag: 4-wave k_verify_prep build -- full GPU suite + smoke, then the
# measurement set bench.py reads (rocprof stats + PMC passes, VALU issue
# calibration, C4 issue pass), as r03p
set -o pipefail
O=gpurun_out/r03ag; mkdir -p $O
export FD_DROPIN_SUMMARY=$O/dropin_c_callers.json
timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -rP > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
bash tools/run_profile.sh r03ag || exit 1
bash tools/run_valu_calib.sh r03ag || exit 1
bash tools/run_c4_issue.sh r03ag || exit 1
