# r06t: one box, depth 16384, 3 tiles, paced x3 at 16 / 20 / 24 M frags/s: this build (quarter-wave gather, ingest
# thread) vs the round-5 gather (FD_VERIFY_SVC_GATHER=wave) vs no ingest thread (FD_VERIFY_SVC_INGEST_THREAD=0)
set -o pipefail
A="--frags,4194304,--tiles,3,--in-depth,16384,--prelay,--rate,16000000+20000000+24000000,--repeat,3,--env,SVC_RUN_REQ_DEPTH=128+SVC_RUN_SLOT_CAP=2048"
bash tools/gpu_session.sh r06t svc:$A svc:$A,--svc-env,FD_VERIFY_SVC_GATHER=wave svc:$A,--svc-env,FD_VERIFY_SVC_INGEST_THREAD=0
