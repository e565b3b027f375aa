# r06n: the gather's share of the GPU at depth 16384, 3 tiles: its grid cap and the DSM's free workgroup slots
set -o pipefail
A="--frags,4194304,--tiles,3,--in-depth,16384,--prelay,--rate,30000000+34000000+38000000,--env,SVC_RUN_REQ_DEPTH=128+SVC_RUN_SLOT_CAP=2048"
bash tools/gpu_session.sh r06n svc:$A svc:$A,--svc-env,FD_VERIFY_SVC_GATHER_WGS=1024 \
  svc:$A,--svc-env,FD_ED25519_HIP_DSM_RESERVE=256 svc:$A,--svc-env,FD_VERIFY_SVC_GATHER_WGS=1024+FD_ED25519_HIP_DSM_RESERVE=256
