# r06r: kernel trace of the GPU tile at depth 16384, 3 tiles, 26 M frags/s offered: the gather's execution time
# against its event bracket (dispatch wait), and what runs beside it
set -o pipefail
bash tools/gpu_session.sh r06r \
  svc:--frags,4194304,--tiles,3,--in-depth,16384,--prelay,--rate,26000000,--env,SVC_RUN_REQ_DEPTH=128+SVC_RUN_SLOT_CAP=2048,--svc-env,SVC_SANDBOX=0,--rocprof,gpurun_out/r06r/prof
