# r06p: the gather with descriptors in LDS and every piece load in flight: service tests (byte-equal to the
# reference tile), then at depth 16384 (svc_bench --in-depth now holds with --prelay): paced runs x3 and the sweep
set -o pipefail
A="--frags,4194304,--tiles,3,--in-depth,16384,--prelay,--rate,24000000+28000000+32000000,--repeat,3,--env,SVC_RUN_REQ_DEPTH=128+SVC_RUN_SLOT_CAP=2048"
S="--frags,4194304,--tiles,3,--depths,16384,--steps,5,--env,SVC_RUN_PRELAY=1+SVC_RUN_REQ_DEPTH=128+SVC_RUN_SLOT_CAP=2048"
bash tools/gpu_session.sh r06p tests:tests/test_gpu_svc_run.py,tests/test_gpu_svc_clients.py,tests/test_gpu_svc_sandbox.py svc:$A sweep:$S
