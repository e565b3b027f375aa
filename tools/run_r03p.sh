#!/bin/bash
# r03p: the measurement set for this kernel build: rocprofv3 kernel stats + PMC passes
# (tools/run_profile.sh), the VALU issue calibration (tools/run_valu_calib.sh), C4's own issue pass
set -o pipefail
bash tools/run_profile.sh r03p || exit 1
bash tools/run_valu_calib.sh r03p || exit 1
bash tools/run_c4_issue.sh r03p || exit 1
