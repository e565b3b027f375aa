#!/bin/bash
# round-4 profile set for the current build: C2 stats + PMC passes, VALU
# issue calibration, C4 issue pass, C4 ingest FETCH/WRITE passes and stats
set -o pipefail
bash tools/run_profile.sh r04p || exit 1
bash tools/run_valu_calib.sh r04p || exit 1
bash tools/run_c4_issue.sh r04p || exit 1
bash tools/gpu_session.sh r04p c4pmc c4stats || exit 1
