"""The verify service's ingest step by step (integration/svc_probe.c), on the
GPU: a segment in the probe's own memory, requests posted by hand through
include/fd_verify_svc.h's tile-side calls, each step under a deadline.

Both ingest forms: the per-request kernel launches (the default) and the
resident IO engine (FD_VERIFY_SVC_IO=io, k_svc_io).  Each must take a frag
request to INGESTED and RESULTS (every zero-byte frag failing its parse, as
fd_txn_parse fails it), retire a flush of host-written entries, and tear down
with the engine stopped."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(REPO, "integration", "_build", "svc_probe")

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["launch", "io"])
def test_probe_steps(mode):
    if not os.path.exists(PROBE):
        pytest.skip("integration/_build/svc_probe not built (build() with /root/reference)")
    env = dict(os.environ, FD_VERIFY_SVC_IO=mode)
    r = subprocess.run(["timeout", "-k", "5", "40", PROBE, "64"], capture_output=True, text=True, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "PROBE OK" in out, out[-3000:]
    assert "64 frags, 64 parse failures" in out, out[-3000:]
    assert "latency: post -> INGESTED" in out, out[-3000:]
