set -o pipefail
mkdir -p gpurun_out/r06k
timeout -k 10 120 tools/_build/hip_host_costs 2000 > gpurun_out/r06k/host_costs.json 2>&1 || exit 3
cat gpurun_out/r06k/host_costs.json
bash tools/gpu_session.sh r06k tests:tests/test_gpu_svc_run.py \
  svc:--frags,4194304,--tiles,3,--in-depth,16384,--prelay,--rate,17000000+22000000+27000000+32000000,--env,SVC_RUN_REQ_DEPTH=128+SVC_RUN_SLOT_CAP=2048 \
  sweep:--frags,4194304,--tiles,3,--depths,16384,--env,SVC_RUN_PRELAY=1+SVC_RUN_REQ_DEPTH=128+SVC_RUN_SLOT_CAP=2048
