#!/bin/bash
# round-4 session q: the verify tile with the GPU-side during_frag copy
# (integration/fd_verify_tile_hip.patch FD_VERIFY_HIP_GPU_COPY): engine and
# patched-tile GPU tests, the tile sweep against the host-copy form, then the
# profile set of this build (tools/r04p_session.sh)
set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_txn_batch.py tests/test_gpu_tile_hip.py tests/test_gpu_txnm.py tests/test_gpu_txn.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 900 python -u tools/tile_bench.py --frags 2097152 --tiles 1,2,4 --in-depth 131072 --configs b4096i2,b4096i4,b8192i4,b8192i4h --timeout 90 --logdir $O/logs > $O/sweep.jsonl 2> $O/sweep.err || { tail -30 $O/sweep.err; exit 1; }
python3 -c "
import json
for l in open('$O/sweep.jsonl'):
    d=json.loads(l)
    if isinstance(d.get('tiles'),list): print(d['config'], d['tile_cnt'], round(d['verifies_per_s']/1e6,2), 'M', 'ovr', d.get('overrun'), 'gpu_ms', d['gpu_ms_per_batch'], 'post', d['regime']['post_processing'])
    else: print(d)
"
bash tools/r04p_session.sh || exit 1
