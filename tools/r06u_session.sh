# r06u: the full GPU suite, smoke and the default bench line on HEAD
set -o pipefail
export FD_BENCH_TILE_LOGDIR=$(pwd)/gpurun_out/r06u/tile_logs
bash tools/gpu_session.sh r06u tests smoke bench
