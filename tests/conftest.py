import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")


def pytest_sessionstart(session):
    """In the build container (where /root/reference exists) build the
    checkers -- the oracle and oracle/_ref, the reference compiled from its
    sources -- before any test looks for them, so the reference-parity tests
    run instead of skipping when the suite is started before build()."""
    if os.path.isdir("/root/reference/src/ballet/ed25519"):
        import subprocess
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(REPO, "oracle"), "oracle", "ref"])
        if os.path.exists(os.path.join(REPO, "firedancer_amd", "libfd_ed25519_hip.so")):
            subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(REPO, "oracle"), "tile"])
            subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(REPO, "integration"), "all"])


@pytest.fixture(scope="session")
def kat():
    with open(os.path.join(HERE, "golden", "kat_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def c2mix():
    d = np.load(os.path.join(HERE, "golden", "c2_mix_4096.npz"))   # allow_pickle=False (default)
    return {k: d[k] for k in d.files}


@pytest.fixture(scope="session")
def verifier():
    import torch
    # GPU tests fail, not skip, without a GPU: a skipped parity test would
    # pass the suite with nothing checked
    assert torch.cuda.is_available(), "GPU test without a usable GPU (torch.cuda.is_available() is False)"
    from firedancer_amd import Verifier
    v = Verifier(device=0, chunk_sigs=1 << 18)
    yield v
    v.close()
