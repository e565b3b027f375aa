#!/bin/bash
# GPU-box script: A/B of k_verify_dsm build variants on one box -- C2 bench
# (one context, so each DSM dispatch is a whole 2^20 batch) plus rocprofv3
# PMC passes for HBM-side bytes, issue slots and held clock per variant.
# Usage: bash tools/run_dsm_variants.sh <tag> <variant> ...   ("" = default build)
export TMPDIR=/tmp
R=$(pwd); T=$1; shift
O=$R/gpurun_out/dsmvar_$T; mkdir -p $O
for v in "$@"; do
  name=${v:-default}
  if [ -n "$v" ]; then export FD_ED25519_HIP_LIB=$v; else unset FD_ED25519_HIP_LIB; fi
  timeout -k 10 200 python3 bench.py --contexts 1 --no-cpu-baseline --steps 10 --warmup 3 > $O/$name.json 2> $O/$name.err || exit $?
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/${name}_p$i -o run -- \
        python3 bench.py --contexts 1 --no-cpu-baseline --steps 2 --warmup 1 > $O/${name}_p$i.out 2> $O/${name}_p$i.err || exit $?
  done
  echo "variant $name done"
done
