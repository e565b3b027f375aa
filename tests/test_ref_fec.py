"""CPU: integration/fd_fec_resolver_hip.patch against the reference's FEC
resolver (src/disco/shred/fd_fec_resolver.c).

The patch lets a caller batch the Merkle-root signature check of new FEC sets
(fd_fec_resolver.c:476) through the GPU (fd_fec_resolver_hip_preverify ->
fd_fec_hip_verify_roots_dev); add_shred takes a verified entry's code for
exactly its own three inputs and verifies anything else on its core.

- Without FD_HAS_HIP the patched resolver preprocesses to the reference's
  own token stream: the patch is inert in a reference build.
- With FD_HAS_HIP it compiles against the reference headers under
  -Wall -Wextra -Werror (integration/Makefile: _build/fec_strict.o).
- integration/fec_run.c feeds the resolver a stream the reference's
  shredder makes (wrong-key slots, corrupted signatures, one corrupted shred
  per 11th set, dropped parity, shuffled windows): the stream is
  deterministic, and the resolver completes, rejects and ignores shreds as
  the faults dictate.
The GPU half (the engine attached, output byte-equal to the reference's) is
tests/test_gpu_fec.py."""
import json
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, "integration", "_build")
REF = "/root/reference"
FEC_TMP = "/tmp/fd_fec_patched_run"
FLAGS = ["-std=c17", "-D_GNU_SOURCE", "-DFD_HAS_HOSTED=1", "-DFD_HAS_INT128=1", "-DFD_HAS_DOUBLE=1",
         "-DFD_HAS_ALLOCA=1", "-DFD_HAS_X86=1", "-DFD_HAS_ATOMIC=1", "-DFD_HAS_THREADS=1", "-march=x86-64"]

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(BUILD, "fec_run_ref")),
                                reason="the FEC drivers need /root/reference (built by build())")


def _tokens(path, extra):
    """the preprocessed token stream of a resolver source, line markers and
    the __FILE__ / __LINE__ of log calls dropped"""
    src = os.path.join(REF, "src", "disco", "shred")
    out = subprocess.run(["gcc", "-E", "-P"] + FLAGS + extra + ["-I" + src, "-I" + os.path.join(REPO, "include"), path],
                         check=True, capture_output=True, text=True).stdout
    return re.sub(r'"[^"]*fd_fec_resolver\.c", \d+', '"F", 0', " ".join(out.split()))


def test_patch_is_inert_without_hip():
    patched = os.path.join(FEC_TMP, "src", "disco", "shred", "fd_fec_resolver.c")
    assert os.path.exists(patched), "integration/Makefile fec target not built"
    ref = _tokens(os.path.join(REF, "src", "disco", "shred", "fd_fec_resolver.c"), [])
    assert _tokens(patched, ["-I" + os.path.dirname(patched)]) == ref
    assert _tokens(patched, ["-I" + os.path.dirname(patched), "-DFD_HAS_HIP=1"]) != ref


def test_patched_resolver_compiles_strict():
    assert os.path.exists(os.path.join(BUILD, "fec_strict.o"))
    nm = subprocess.run(["nm", os.path.join(BUILD, "fec_strict.o")], check=True, capture_output=True, text=True).stdout
    for sym in ("fd_fec_resolver_hip_attach", "fd_fec_resolver_hip_preverify", "fd_fec_resolver_hip_stats",
                "fd_fec_resolver_add_shred"):
        assert f" T {sym}" in nm, sym
    assert " U fd_fec_hip_verify_roots_dev" in nm


def _run(tmp_path, exe, sets, seed, window, name):
    out = str(tmp_path / name)
    p = subprocess.run([os.path.join(BUILD, exe), out, str(sets), str(seed), str(window)], capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1]), open(out, "rb").read()


def test_reference_resolver_on_the_shredder_stream(tmp_path):
    r, b = _run(tmp_path, "fec_run_ref", 200, 0x5eedfec, 512, "a.bin")
    r2, b2 = _run(tmp_path, "fec_run_ref", 200, 0x5eedfec, 512, "b.bin")
    assert b == b2                                               # deterministic
    assert {k: v for k, v in r.items() if k != "resolver_s"} == {k: v for k, v in r2.items() if k != "resolver_s"}
    assert r["hip"] == 0 and r["sets"] == 200
    assert r["rejected"] + r["ignored"] + r["okay"] + r["completes"] == r["shreds"]
    # every 7th slot is signed by another key and every 13th set carries a bad signature:
    # those never complete; the others do (no data shred is dropped)
    assert 0.6 * r["sets"] < r["completes"] < r["sets"] and r["rejected"] > 0
    _, b3 = _run(tmp_path, "fec_run_ref", 200, 0x5eedfed, 512, "c.bin")
    assert b3 != b
