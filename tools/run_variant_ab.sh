#!/bin/bash
# GPU-box script: GPU parity tests on a library variant, then an A/B bench
# alternating it with the default build.
#   bash tools/run_variant_ab.sh <variant>   (firedancer_amd/libfd_ed25519_hip_<variant>.so)
set -o pipefail
mkdir -p gpurun_out
V=${1:?variant}
FD_ED25519_HIP_LIB=$PWD/firedancer_amd/libfd_ed25519_hip_$V.so timeout -k 10 600 \
    python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_$V.log 2>&1 \
    || { tail -40 gpurun_out/pytest_$V.log; exit 1; }
tail -2 gpurun_out/pytest_$V.log
bash tools/run_ab.sh default $V default $V
