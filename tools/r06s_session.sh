# r06s: gathers alternating over two ingest streams (default) vs one (FD_VERIFY_SVC_ING_STREAMS=1), depth 16384,
# 3 tiles, paced x2 at 24 / 28 / 32 M frags/s; the sweep with two; service tests
set -o pipefail
A="--frags,4194304,--tiles,3,--in-depth,16384,--prelay,--rate,24000000+28000000+32000000,--repeat,2,--env,SVC_RUN_REQ_DEPTH=128+SVC_RUN_SLOT_CAP=2048"
S="--frags,4194304,--tiles,3,--depths,16384,--steps,5,--env,SVC_RUN_PRELAY=1+SVC_RUN_REQ_DEPTH=128+SVC_RUN_SLOT_CAP=2048"
bash tools/gpu_session.sh r06s tests:tests/test_gpu_svc_run.py,tests/test_gpu_svc_clients.py svc:$A svc:$A,--svc-env,FD_VERIFY_SVC_ING_STREAMS=1 sweep:$S
