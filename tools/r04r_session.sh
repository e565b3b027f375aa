#!/bin/bash
# round-4 session r: tile sweep, GPU-side during_frag (producer margin for held frags) vs host copy
set -o pipefail
O=gpurun_out/r04r; mkdir -p $O
timeout -k 10 1000 python -u tools/tile_bench.py --frags 2097152 --tiles 1,2,4 --in-depth 131072 --configs b4096i2,b8192i2,b8192i3,b8192i4,b8192i4h --timeout 90 --logdir $O/logs > $O/sweep.jsonl 2> $O/sweep.err || { tail -30 $O/sweep.err; exit 1; }
python3 -c "
import json
for l in open('$O/sweep.jsonl'):
    d=json.loads(l)
    if isinstance(d.get('tiles'),list): print(d['config'], d['tile_cnt'], round(d['verifies_per_s']/1e6,2), 'M', 'frags/s', round(d['frags_per_s']/1e6,2), 'ovr', d.get('overrun'), 'gpu_ms', d['gpu_ms_per_batch'], 'post', d['regime']['post_processing'], 'cu', d['regime']['caught_up'], 'depth', d['in_depth'])
    else: print(d)
"
