#!/usr/bin/env python3
"""one line per service-mode run of a tools/svc_bench.py JSONL file"""
import json
import sys
for path in sys.argv[1:]:
    for l in open(path):
        r = json.loads(l)
        if not isinstance(r.get("tiles"), list):
            continue
        busy = [x.get("busy_s", {}) for x in r["tiles"]]
        b = {k: round(max(x.get(k, 0) for x in busy), 3) for k in ("publish", "pass", "flush", "post")}
        sv = r["svc"]
        print(f"T{r['tile_cnt']} {r['verifies_per_s']/1e6:6.1f} M/s {r['frags_per_s']/1e6:5.1f} Mfr/s {r['seconds']:.3f}s "
              f"launch {sv['launches']} ({sv['frags']/max(sv['launches'],1)/1e3:.0f}K fr) gpu {sv['gpu_s']:.3f}s "
              f"flush {sv['flushes']} ({sv['flushed_frags']/max(sv['flushes'],1):.0f} fr) spans {sv['spans']} "
              f"reg {r['regime']} tile-busy {b} ovr {r['overrun']}/{r['lapped']} lat {r['latency']['p50_us']}/{r['latency']['p99_us']}"
              + (f" slots {sv['slots']}" if "slots" in sv else ""))
