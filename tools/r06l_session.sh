# r06l: the full GPU suite, smoke and the default bench line on HEAD (ingest thread)
set -o pipefail
export FD_BENCH_TILE_LOGDIR=$(pwd)/gpurun_out/r06l/tile_logs
bash tools/gpu_session.sh r06l tests smoke bench
