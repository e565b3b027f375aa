"""The profile summaries bench.py prices its roofline with must describe the
kernels of the library in the tree: each summary records the gfx950
machine-code hashes of k_verify_dsm / k_verify_prep
(firedancer_amd/kernel_hash.py; the C4 ingest summary also k_txnm_batch<16>),
and a kernel change without a fresh measurement set (tools/run_profile.sh,
run_valu_calib.sh, run_c4_issue.sh, gpu_session.sh c4pmc)
fails here instead of silently reporting another build's counters.
CPU-only: reads the built library's ELF, launches nothing."""
import json
import os

import pytest

import bench
from firedancer_amd.kernel_hash import engine_kernel_hashes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("name", [bench.PMC_SUMMARY, bench.ISSUE_SUMMARY, bench.ISSUE_SUMMARY_C4])
def test_profile_summary_matches_built_kernels(name):
    lib = os.path.join(REPO, "firedancer_amd", "libfd_ed25519_hip.so")
    assert os.path.exists(lib), "build the engine first (__graft_entry__.build())"
    with open(os.path.join(REPO, "profiles", name)) as f:
        summary = json.load(f)
    want = summary.get("kernel_sha") or {}
    assert set(want) >= {"k_verify_dsm", "k_verify_prep"}, f"{name} records no kernel hashes"
    have = engine_kernel_hashes()
    for k in ("k_verify_dsm", "k_verify_prep"):
        assert want[k] == have[k], (f"profiles/{name} was measured on another {k} build "
                                    f"({want[k]} vs {have[k]}): rerun the profile set")
    assert bench.profile_build_check(summary)["profile_matches_build"] is True


def test_c4_ingest_summary_matches_built_kernel():
    """profiles/PMC_SUMMARY_C4 (the C4 bench's FETCH/WRITE passes,
    tools/txnm_pmc_summary.py) priced k_txnm_batch<16> of this build."""
    with open(os.path.join(REPO, "profiles", bench.PMC_SUMMARY_C4)) as f:
        summary = json.load(f)
    want = summary.get("kernel_sha") or {}
    have = engine_kernel_hashes(names=("k_verify_dsm", "k_verify_prep", "k_txnm_batch<16>"))
    for k in ("k_verify_dsm", "k_verify_prep", "k_txnm_batch<16>"):
        assert want.get(k) == have[k], (f"profiles/{bench.PMC_SUMMARY_C4} was measured on another {k} build "
                                        f"({want.get(k)} vs {have[k]})")
    kb = summary["kernels"]["k_txnm_batch"]
    assert kb["algorithmic_bytes_per_launch"] > 0 and 1.0 <= kb["traffic_ratio"] < 2.0
