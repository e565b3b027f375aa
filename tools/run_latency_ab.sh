#!/bin/bash
# GPU-box script: drop-in per-call latency (tools/bench_latency.py) for the
# default build and library variants, alternating.
# Usage: bash tools/run_latency_ab.sh <tag> <variant>...
T=$1; shift; O=gpurun_out/latab_$T; mkdir -p $O
for rep in 1 2; do
  for v in default "$@"; do
    if [ $v != default ]; then export FD_ED25519_HIP_LIB=$PWD/firedancer_amd/libfd_ed25519_hip_$v.so; else unset FD_ED25519_HIP_LIB; fi
    timeout -k 10 200 python tools/bench_latency.py 1000 > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -5 $O/${v}_$rep.err; exit 1; }
    echo "$v $rep $(cat $O/${v}_$rep.json)"
  done
done
