"""firedancer_amd: MI355X (gfx950) ed25519 batch signature verification for the
Firedancer verify path (drop-in for src/ballet/ed25519/fd_ed25519.h).

The product is the C-ABI library libfd_ed25519_hip.so (include/fd_ed25519_hip.h);
this package holds its sources (csrc/), its build, the Python mirrors of the
reference interfaces (ed25519.py: fd_ed25519.h; verify_tile.py: the verify
tile's GPU batch path; replay.py: fd_executor_txn_verify, the FEC root check
and the ed25519 precompile) and the synthetic workloads (workload.py,
txn_workload.py)."""
from .ed25519 import (FD_ED25519_ERR_MSG, FD_ED25519_ERR_PUBKEY, FD_ED25519_ERR_SIG,  # noqa: F401
                      FD_ED25519_SUCCESS, ERRMODE_AVX512, ERRMODE_REF, Verifier, fd_ed25519_strerror,
                      fd_ed25519_verify, fd_ed25519_verify_batch_single_msg)
