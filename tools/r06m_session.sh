# r06m: the ingest thread's setup before the sandbox: trap-mode service runs (any refused call named in svc.err),
# then the default bench line
set -o pipefail
export FD_BENCH_TILE_LOGDIR=$(pwd)/gpurun_out/r06m/tile_logs
bash tools/gpu_session.sh r06m env:SVC_SANDBOX=trap \
  svc:--frags,4194304,--tiles,3,--in-depth,16384,--prelay,--rate,24000000+28000000+32000000,--repeat,2,--env,SVC_RUN_REQ_DEPTH=128+SVC_RUN_SLOT_CAP=2048 || exit $?
grep -rh "seccomp trap" gpurun_out/r06m/svc_logs_2 | sort | uniq -c | head; echo "traps listed above (none: clean)"
unset SVC_SANDBOX
bash tools/gpu_session.sh r06m bench
