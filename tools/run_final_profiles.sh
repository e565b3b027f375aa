#!/bin/bash
# GPU-box script: the round's final measurement set on one box: rocprofv3
# kernel stats + PMC passes (run_profile.sh), the VALU issue calibration
# (run_valu_calib.sh), and a one-minute C2 run with power/clock samples.
# Usage: bash tools/run_final_profiles.sh <tag>
T=${1:?tag}
bash tools/run_profile.sh $T || exit 1
bash tools/run_valu_calib.sh $T || exit 1
bash tools/run_power.sh power_$T 8000 || exit 1
