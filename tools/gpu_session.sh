#!/bin/bash
# GPU-box session runner: one parameterised script for the measurement steps
# the per-session run_*.sh scripts used to spell out one by one.
#
# Usage: bash tools/gpu_session.sh <tag> <step> [<step> ...]
#   -> gpurun_out/<tag>/...   (stops at the first failing step)
#
# Steps (arguments after ':' are passed on, ',' separates them, '+' stands for
# a ',' inside one argument: --tiles,1+2+4 is --tiles 1,2,4):
#   tests[:files]      pytest -m gpu on the given test files (default: all)
#   bench[:args]       python bench.py <args>                  -> bench_<n>.json
#   c4[:args]          python bench.py --config c4 <args>       -> c4_<n>.json
#   ab[:ENV=V,...]     C4 bench with extra environment (A/B)    -> ab_<n>.json
#   stats[:args]       rocprofv3 --kernel-trace --stats of bench.py --contexts 1 <args>
#   c4stats[:args]     the same over the C4 bench (one tile, serialised dispatches)
#   pmc                PMC passes over bench.py --contexts 1: VALU issue group,
#                      SQ group, FETCH_SIZE, WRITE_SIZE, TCC/GRBM (one pass each)
#   c4pmc[:args]       VALU issue + FETCH_SIZE + WRITE_SIZE passes over the C4 bench
#   tile[:args]        python tools/tile_bench.py <args>        -> tile_<n>.json
#   replay[:args]      python tools/replay_block_bench.py <args> -> replay_<n>.json
#   profile            the profile set bench.py prices its rooflines with, for this build:
#                      tools/run_profile.sh, run_valu_calib.sh and run_c4_issue.sh (tag <tag>),
#                      then the c4pmc and c4stats steps; summarise with tools/pmc_summary.py,
#                      valu_calib_summary.py, c4_issue_summary.py, txnm_pmc_summary.py
#   smoke              __graft_entry__.smoke()
#   svc[:args]         python tools/svc_bench.py <args>         -> svc_<n>.jsonl (the service-mode stage)
#   sweep[:args]       python tools/svc_link_sweep.py <args>    -> sweep_<n>.jsonl, table in sweep_<n>.err
#   env:K=V,...        export K=V for the steps after it (e.g. SVC_BENCH_TILE_EXE=integration/_build/svc_tile_run_d2)
# Round-5 service sessions, as steps (their one-off scripts tools/r05*_session.sh are in git history):
#   the DSM reserve A/B (r05aq): svc:--frags,4194304,--tiles,2+3,--repeat,2,--prelay,--env,SVC_RUN_REQ_DEPTH=8
#                                svc:...,--svc-env,FD_ED25519_HIP_DSM_RESERVE=192
#   the link sweep (r05al):      sweep:--tiles,2,--depths,16384+65536+262144,--env,SVC_RUN_REQ_DEPTH=64+SVC_RUN_SLOT_CAP=8192
# Round-4 sessions, as steps: replay/tile tests + tile sweep (r04n) =
#   tests:tests/test_gpu_replay_block.py,tests/test_gpu_replay.py,tests/test_gpu_txn_batch.py,tests/test_gpu_tile_hip.py
#   replay:--txns,16384+98039,--sched  tile:--frags,2097152,--tiles,1+2+4,--configs,b8192i4+b8192i4h
# the link-walk bound (r04o): tile:--walk,--tiles,1+2+4,--configs,b8192i4
# range mode (r04w): tile:--frags,2097152,--tiles,1+2+4,--configs,b8192i3r+b8192i3+b4096i3r
# (It replaces the round-3 per-session scripts tools/run_r03*.sh and the
# one-off A/B runners; they are in git history before this file's commit.)
# Every GPU step runs under its own timeout; a failure ends the session.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
T=${1:?tag}; shift
O=$R/gpurun_out/$T
mkdir -p $O
n=0
VALU_G="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
SQ_G="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"

fail() { echo "step $1 failed (rc=$2)"; [ -n "$3" ] && tail -40 "$3"; exit $2; }
args_of() { local a="${1#*:}"; [ "$a" = "$1" ] && a=""; a="${a//,/ }"; echo "${a//+/,}"; }

pmc_pass() {   # <name> <counters> <cmd...>
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/$name -o run -- "$@" \
      > $O/$name.out 2> $O/$name.err || fail $name $? $O/$name.err
  echo "pmc $name ok"
}

for step in "$@"; do
  n=$((n+1))
  a=$(args_of "$step")
  case "${step%%:*}" in
    tests)
      timeout -k 10 1500 python -u -m pytest ${a:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
          -p no:cacheprovider > $O/pytest_$n.txt 2>&1 || fail tests $? $O/pytest_$n.txt
      tail -3 $O/pytest_$n.txt ;;
    bench)
      timeout -k 10 600 python bench.py $a > $O/bench_$n.json 2> $O/bench_$n.err || fail bench $? $O/bench_$n.err
      cut -c1-400 $O/bench_$n.json ;;
    c4)
      timeout -k 10 900 python bench.py --config c4 $a > $O/c4_$n.json 2> $O/c4_$n.err || fail c4 $? $O/c4_$n.err
      python3 -c "import json,sys; d=json.load(open('$O/c4_$n.json')); print('c4', d['value'], (d.get('pcie_inclusive') or {}).get('value'), d.get('batch_gpu_ms'))" ;;
    ab)
      timeout -k 10 900 env $a python bench.py --config c4 --no-cpu-baseline --c4-pcie-steps 4 \
          > $O/ab_$n.json 2> $O/ab_$n.err || fail ab $? $O/ab_$n.err
      python3 -c "import json; d=json.load(open('$O/ab_$n.json')); print('ab [$a]', d['value'], d.get('batch_gpu_ms'))" ;;
    stats)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$n -o run -- \
          python3 bench.py --contexts 1 --no-c4 $a > $O/stats_$n.json 2> $O/stats_$n.err || fail stats $? $O/stats_$n.err
      echo "stats ok" ;;
    c4stats)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4stats_$n -o run -- \
          python3 bench.py --config c4 --tiles 1 --no-cpu-baseline --steps 3 --warmup 1 --c4-pcie-steps 1 $a \
          > $O/c4stats_$n.json 2> $O/c4stats_$n.err || fail c4stats $? $O/c4stats_$n.err
      echo "c4stats ok" ;;
    pmc)
      B="python3 bench.py --contexts 1 --no-c4 --no-cpu-baseline --steps 2 --warmup 1"
      pmc_pass pmc_valu "$VALU_G" $B
      pmc_pass pmc_sq "$SQ_G" $B
      pmc_pass pmc_fetch "FETCH_SIZE" $B
      pmc_pass pmc_write "WRITE_SIZE" $B
      pmc_pass pmc_tcc "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" $B ;;
    c4pmc)
      B="python3 bench.py --config c4 --tiles 1 --no-cpu-baseline --steps 2 --warmup 1 --c4-pcie-steps 1 $a"
      pmc_pass c4pmc_valu "$VALU_G" $B
      pmc_pass c4pmc_fetch "FETCH_SIZE" $B
      pmc_pass c4pmc_write "WRITE_SIZE" $B ;;
    tile)
      timeout -k 10 900 python3 tools/tile_bench.py $a > $O/tile_$n.json 2> $O/tile_$n.err || fail tile $? $O/tile_$n.err
      tail -c 600 $O/tile_$n.json ;;
    replay)
      timeout -k 10 600 python3 -u tools/replay_block_bench.py $a > $O/replay_$n.json 2> $O/replay_$n.err \
          || fail replay $? $O/replay_$n.err
      cut -c1-600 $O/replay_$n.json ;;
    profile)
      bash tools/run_profile.sh $T || fail profile $?
      bash tools/run_valu_calib.sh $T || fail valu $?
      bash tools/run_c4_issue.sh $T || fail c4issue $?
      B="python3 bench.py --config c4 --tiles 1 --no-cpu-baseline --steps 2 --warmup 1 --c4-pcie-steps 1"
      pmc_pass c4pmc_valu "$VALU_G" $B
      pmc_pass c4pmc_fetch "FETCH_SIZE" $B
      pmc_pass c4pmc_write "WRITE_SIZE" $B
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4stats_$n -o run -- \
          python3 bench.py --config c4 --tiles 1 --no-cpu-baseline --steps 3 --warmup 1 --c4-pcie-steps 1 \
          > $O/c4stats_$n.json 2> $O/c4stats_$n.err || fail c4stats $? $O/c4stats_$n.err
      echo "profile set ok" ;;
    svc)
      timeout -k 10 900 python3 -u tools/svc_bench.py --logdir $O/svc_logs_$n $a > $O/svc_$n.jsonl 2> $O/svc_$n.err \
          || fail svc $? $O/svc_$n.err
      python3 -c "
import json
for l in open('$O/svc_$n.jsonl'):
    d = json.loads(l)
    if 'tiles' in d and isinstance(d['tiles'], list):
        print('svc', d['tile_cnt'], round(d['verifies_per_s']/1e6, 2), 'M v/s', round(d['frags_per_s']/1e6, 2), 'M f/s lost', d['overrun'] + d['lapped'] + d.get('unseen', 0), 'p99', d['latency']['p99_us'])
" ;;
    sweep)
      timeout -k 10 1100 python3 -u tools/svc_link_sweep.py --logdir $O/sweep_logs_$n $a > $O/sweep_$n.jsonl \
          2> $O/sweep_$n.err || fail sweep $? $O/sweep_$n.err
      grep depth_summary $O/sweep_$n.jsonl | cut -c1-400 ;;
    env)
      for kv in $a; do export "$kv"; done; echo "env $a" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || fail smoke $? $O/smoke.txt
      tail -2 $O/smoke.txt ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
