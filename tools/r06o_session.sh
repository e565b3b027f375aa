# r06o: losses at 20-28 M frags/s while 30-38 M runs lose none (r06m, r06n): repeated mid-rate runs and the
# bench's bisection, with and without CUs kept free of verify kernels for the gather and flush kernels
set -o pipefail
E="--env,SVC_RUN_REQ_DEPTH=128+SVC_RUN_SLOT_CAP=2048"
A="--frags,4194304,--tiles,3,--in-depth,16384,--prelay,--rate,22000000+24000000+26000000,--repeat,3,$E"
S="--frags,4194304,--tiles,3,--depths,16384,--steps,5,--env,SVC_RUN_PRELAY=1+SVC_RUN_REQ_DEPTH=128+SVC_RUN_SLOT_CAP=2048"
bash tools/gpu_session.sh r06o svc:$A sweep:$S \
  svc:$A,--svc-env,FD_VERIFY_SVC_FREE_CUS=16 sweep:$S,--svc-env,FD_VERIFY_SVC_FREE_CUS=16 \
  svc:$A,--svc-env,FD_VERIFY_SVC_FREE_CUS=32 sweep:$S,--svc-env,FD_VERIFY_SVC_FREE_CUS=32
