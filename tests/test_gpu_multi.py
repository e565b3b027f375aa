"""GPU: the sharded (N>1) verify path with real kernels.

1. Two fresh rank processes (tests/multi_rank_worker.py, gloo group, one
   verify context each on GPU 0) verify their shard_bounds halves of one
   2^23-signature C2-mix batch and all-gather the verdict bitmap; it must
   equal a single-process whole-batch pass, whose codes must equal the CPU
   oracle on an 8K sample (BASELINE configs[4]).
2. bench.py's own N>1 code (torch.distributed.run, max-over-ranks time,
   all-reduced signature count, C5 strong-scaling shards) at world size 2,
   rehearsed with --dist-backend gloo because both ranks share the box's one
   GPU (RCCL refuses two ranks on one device).

The ranks are started as child processes of this (GPU-initialised) test
process with subprocess, never by exec.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_two_ranks_shard_and_gather(tmp_path):
    n, world = 1 << 23, 2
    port = _free_port()
    procs, outs = [], []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out = tmp_path / f"rank{r}.json"
        outs.append(out)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "multi_rank_worker.py"), str(n), str(out)],
                                      env=env, cwd=REPO))
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=240))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert rcs == [0] * world, rcs
    res = [json.load(open(o)) for o in outs]
    assert res[0]["lo"] == 0 and res[-1]["hi"] == n and res[0]["hi"] == res[1]["lo"]
    r0 = res[0]
    assert r0["bitmap_equal"], r0
    assert r0["bitmap_is_codes"] and r0["codes_set"], r0
    assert r0["oracle_sample_equal"], r0
    assert 0.75 < r0["accept"] < 0.83, r0


@pytest.mark.gpu
def test_bench_world2_c5_gloo(tmp_path):
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
           "--config", "c5", "--sigs", str(1 << 21), "--steps", "2", "--warmup", "1",
           "--dist-backend", "gloo", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["config"]["config_id"] == "c5"
    assert d["value"] > 0 and d["steps"] == 2
    assert str(1 << 22) in d["config"]["workload"]          # n_all all-reduced over both ranks
