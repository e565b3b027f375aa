"""GPU: the shred FEC resolver with integration/fd_fec_resolver_hip.patch and
the engine attached (integration/fec_run.c, _build/fec_run) against the
same resolver built without FD_HAS_HIP -- the reference's add_shred
(_build/fec_run_ref) -- on streams the reference's own shredder makes:
wrong-key slots, corrupted signatures, a corrupted shred per 11th set,
dropped parity shreds, shuffled windows.

- Every shred's add_shred outcome and every completed set (slot,
  fec_set_idx, Merkle root, a hash of its data and parity shreds) are
  byte-equal to the reference's, at windows of 64, 512 and 4096 shreds.
- Every root the GPU verified gives the code the reference's own
  fd_ed25519_verify gives on the same root, signature and leader key
  (the driver checks each one; errmode of the reference's portable build).
- add_shred takes the GPU's code for almost every first shred: core
  verifies are at most 1% of the table hits."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, "integration", "_build")


def _run(tmp_path, exe, sets, seed, window, name):
    assert os.path.exists(os.path.join(BUILD, exe)), "integration/_build missing: run build() with /root/reference"
    out = str(tmp_path / name)
    p = subprocess.run([os.path.join(BUILD, exe), out, str(sets), str(seed), str(window)], capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1]), open(out, "rb").read()


@pytest.mark.parametrize("window", [64, 512, 4096])
def test_gpu_roots_give_the_reference_outcomes(tmp_path, window):
    sets, seed = 1024, 0x5eedfec + window
    ref, rb = _run(tmp_path, "fec_run_ref", sets, seed, window, "ref.bin")
    gpu, gb = _run(tmp_path, "fec_run", sets, seed, window, "gpu.bin")
    print(json.dumps({"window": window, "ref": ref, "gpu": gpu}))
    assert gpu["hip"] == 1 and ref["hip"] == 0
    assert gb == rb
    for k in ("shreds", "sets", "rejected", "ignored", "okay", "completes"):
        assert gpu[k] == ref[k], k
    assert gpu["roots_checked"] == gpu["roots_verified"] > 0 and gpu["code_mismatch"] == 0
    assert gpu["table_hits"] > 0 and gpu["core_verifies"] <= 0.01 * gpu["table_hits"]
