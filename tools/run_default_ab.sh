#!/bin/bash
# GPU-box script: full GPU parity suite on the default build, then a C2 A/B
# bench alternating it with a variant (firedancer_amd/libfd_ed25519_hip_<variant>.so).
set -o pipefail
mkdir -p gpurun_out
V=${1:?variant}
timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 \
    || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash tools/run_ab.sh default $V default $V default $V
