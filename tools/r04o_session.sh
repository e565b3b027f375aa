#!/bin/bash
# round-4 session: default bench (C2 + C4 sub-object) wall time, C4 ingest
# A/B (fused FB16 / FB8 / split), drop-in lat_max A/B, tile link walk
set -o pipefail
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_precheck_fail.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_precheck.txt 2>&1 || { tail -30 $O/pytest_precheck.txt; exit 1; }
tail -2 $O/pytest_precheck.txt
t0=$(date +%s%N)
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
t1=$(date +%s%N); echo "bench wall_s $(( (t1-t0)/1000000000 ))" | tee $O/bench_wall.txt
cut -c1-300 $O/bench.json
for v in fused:FD_VERIFY_HIP_FB=16 fb8:FD_VERIFY_HIP_FB=8 split:FD_VERIFY_HIP_INGEST=split; do
  n=${v%%:*}; e=${v#*:}
  timeout -k 10 600 env $e python bench.py --config c4 --no-cpu-baseline --c4-pcie-steps 2 > $O/c4_$n.json 2> $O/c4_$n.err || { tail -20 $O/c4_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4_$n.json')); print('$n', d['value'], d.get('batch_gpu_ms'), (d.get('ingest_roofline') or {}).get('achieved'))"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin_concurrent.py -m gpu -x -q -s --timeout 200 --timeout-method thread > $O/dropin_default.txt 2>&1 || { tail -20 $O/dropin_default.txt; exit 1; }
FD_ED25519_HIP_DROPIN_LAT_MAX=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin_concurrent.py -m gpu -x -q -s --timeout 200 --timeout-method thread > $O/dropin_lat32.txt 2>&1 || { tail -20 $O/dropin_lat32.txt; exit 1; }
grep -h "sig" $O/dropin_default.txt $O/dropin_lat32.txt | cut -c1-300 | head -12
timeout -k 10 600 python -u tools/tile_bench.py --frags 2097152 --tiles 1,2,4 --walk --configs b8192i4 --timeout 90 --logdir $O/logs > $O/walk.jsonl 2> $O/walk.err || { tail -20 $O/walk.err; exit 1; }
cut -c1-300 $O/walk.jsonl
timeout -k 10 300 python -u tools/replay_block_bench.py --txns 16384,98039 --sched > $O/replay.jsonl 2> $O/replay.err || { tail -20 $O/replay.err; exit 1; }
cut -c1-700 $O/replay.jsonl
