#!/bin/bash
# GPU-box script: A/B of build variants on the SHA-512 paths: the CAVP /
# edge tests, C2 and C4 benches, batched SHA-512 throughput.
# Usage: bash tools/run_ab_c4.sh <tag> <variant>...   ("" = default build)
T=$1; shift; O=gpurun_out/abc4_$T; mkdir -p $O
for v in "$@"; do
  if [ -n "$v" ]; then export FD_ED25519_HIP_LIB=$v; else unset FD_ED25519_HIP_LIB; fi
  n=$(basename ${v:-default} .so)
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sha512_cavp.py \
      tests/test_gpu_sha512.py tests/test_gpu_txnm.py -m gpu > $O/pytest_$n.log 2>&1 || { echo "pytest $n failed"; tail -20 $O/pytest_$n.log; exit 1; }
  tail -1 $O/pytest_$n.log
done
for rep in 1 2; do
  for v in "$@"; do
    if [ -n "$v" ]; then export FD_ED25519_HIP_LIB=$v; else unset FD_ED25519_HIP_LIB; fi
    n=$(basename ${v:-default} .so)
    timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_${n}_$rep.json 2> $O/c2_${n}_$rep.err || exit 1
    timeout -k 10 400 python bench.py --config c4 --steps 8 --warmup 2 --no-cpu-baseline > $O/c4_${n}_$rep.json 2> $O/c4_${n}_$rep.err || exit 1
    python3 -c "
import json; a=json.load(open('$O/c2_${n}_$rep.json')); b=json.load(open('$O/c4_${n}_$rep.json'))
print('$n', $rep, 'c2', round(a['value']/1e6,2), 'prep', a['pipeline']['prep_ms'], 'c4', round(b['value']/1e6,2), 'c4 prep', b['roofline']['prep_ms_per_batch'], 'pcie', round(b['pcie_inclusive']['value']/1e6,2))"
  done
done
for v in "$@"; do
  if [ -n "$v" ]; then export FD_ED25519_HIP_LIB=$v; else unset FD_ED25519_HIP_LIB; fi
  timeout -k 10 300 python tools/bench_sha512.py > $O/sha_$(basename ${v:-default} .so).jsonl 2>/dev/null || exit 1
  python3 -c "
import json
for l in open('$O/sha_$(basename ${v:-default} .so).jsonl'): d=json.loads(l); print('${v:-default}', 'sha', d['msg_bytes'], d['msg_GBps'], d['sample_equal_hashlib'])"
done
