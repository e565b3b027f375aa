"""CPU: the C-ABI library loads and exports every symbol include/*.h declares
(no compute calls without a GPU)."""
import ctypes
import os
import re
import subprocess

from firedancer_amd import ed25519, replay, sha512, verify_tile
from firedancer_amd.build import LIB, build

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(header="fd_ed25519_hip.h"):
    hdr = open(os.path.join(REPO, "include", header)).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    names = set(re.findall(r"\b(fd_\w*)\s*\(", hdr))
    inline = set(re.findall(r"static\s+inline\s+\w+\s+(fd_\w+)\s*\(", hdr))   # header-only helpers
    return names - inline


def test_build_and_exports():
    build()
    assert os.path.exists(LIB)
    assert declared_functions("fd_ed25519_hip.h") == set(ed25519.EXPORTS)
    assert declared_functions("fd_verify_hip.h") == set(verify_tile.EXPORTS)
    assert declared_functions("fd_replay_hip.h") == set(replay.EXPORTS)
    assert declared_functions("fd_sha512_hip.h") == set(sha512.EXPORTS)
    names = set(ed25519.EXPORTS) | set(verify_tile.EXPORTS) | set(replay.EXPORTS) | set(sha512.EXPORTS)
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = set(re.findall(r" T (\w+)", out))
    assert names <= exported, names - exported
    lib = ctypes.CDLL(LIB)
    for n in names:
        assert getattr(lib, n)


def test_strerror_matches_reference():
    # fd_ed25519_user.c:312-322 (no GPU needed: pure host function)
    assert ed25519.fd_ed25519_strerror(0) == "success"
    assert ed25519.fd_ed25519_strerror(-1) == "bad signature"
    assert ed25519.fd_ed25519_strerror(-2) == "bad public key"
    assert ed25519.fd_ed25519_strerror(-3) == "bad message"
    assert ed25519.fd_ed25519_strerror(7) == "unknown"


def test_no_reference_or_oracle_in_product():
    """The product package must not load the oracle or read /root/reference."""
    pkg = os.path.join(REPO, "firedancer_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h")):
                s = open(os.path.join(root, f)).read()
                assert "liboracle" not in s and "oracle_lib" not in s and "/root/reference" not in s, f


def test_headers_compile_and_link_as_c(tmp_path):
    """The boundary is a C ABI: a C11 translation unit (as the reference's C
    tiles would be) includes all four headers next to the system headers
    with -Wall -Wextra -Werror, takes the address of every declared function,
    links against the library and runs (no GPU call)."""
    build()
    names = set()
    for h in ("fd_ed25519_hip.h", "fd_verify_hip.h", "fd_replay_hip.h", "fd_sha512_hip.h"):
        names |= declared_functions(h)
    src = ['#include <stdio.h>', '#include <stdint.h>', '#include <sys/types.h>',
           '#include "fd_ed25519_hip.h"', '#include "fd_verify_hip.h"', '#include "fd_replay_hip.h"',
           '#include "fd_sha512_hip.h"',
           'static void * const fns[] = {']
    src += ['  (void *)%s,' % n for n in sorted(names)]
    src += ['};', 'int main( void ) { printf( "%d\\n", (int)(sizeof(fns)/sizeof(fns[0])) ); return 0; }']
    c = tmp_path / "abi.c"
    c.write_text("\n".join(src) + "\n")
    exe = tmp_path / "abi"
    libdir = os.path.dirname(LIB)
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(REPO, "include"),
                           str(c), "-L", libdir, "-lfd_ed25519_hip", "-Wl,-rpath-link,/opt/rocm/lib",
                           "-Wl,-rpath," + libdir, "-o", str(exe)])
    out = subprocess.check_output([str(exe)]).decode().strip()
    assert int(out) == len(names)


def test_kernel_hashes_found():
    """firedancer_amd/kernel_hash.py finds the bulk kernels' gfx950 code in the
    built library (bench.py uses it to tell whether the committed profile
    summaries measured this build)."""
    from firedancer_amd.kernel_hash import engine_kernel_hashes
    h = engine_kernel_hashes()
    assert set(h) == {"k_verify_dsm", "k_verify_prep"}, h
    assert all(len(v) == 16 and int(v, 16) >= 0 for v in h.values())


def test_range_frag_cnt_matches(tmp_path):
    """fd_verify_hip_range_frag_cnt (include/fd_verify_hip.h, the patched
    tile's count of its round robin share of a seq range) against its Python
    mirror and a brute-force count, seqs near 0 and near 2^40."""
    import itertools
    grid = [(s0, cnt, rr, idx) for s0, cnt, rr in itertools.product((0, 1, 5, 2**40 + 3), (0, 1, 2, 7, 64, 1000),
                                                                      (1, 2, 3, 6, 16))
            for idx in (0, rr - 1, rr // 2, rr)]                     # idx == rr: an out of range index (0)
    src = ['#include <stdio.h>', '#include "fd_verify_hip.h"', 'static const unsigned long g[][4] = {']
    src += ['  { %dUL, %dUL, %dUL, %dUL },' % t for t in grid]
    src += ['};', 'int main( void ) {', '  for( unsigned long i=0; i<sizeof(g)/sizeof(g[0]); i++ )',
            '    printf( "%lu\\n", fd_verify_hip_range_frag_cnt( g[i][0], g[i][1], g[i][2], g[i][3] ) );',
            '  return 0;', '}']
    c = tmp_path / "rc.c"
    c.write_text("\n".join(src) + "\n")
    exe = tmp_path / "rc"
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(REPO, "include"),
                           str(c), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).decode().split()]
    for (s0, cnt, rr, idx), g in zip(grid, got):
        brute = sum(1 for q in range(s0, s0 + cnt) if q % rr == idx) if idx < rr else 0
        assert g == brute == verify_tile.range_frag_cnt(s0, cnt, rr, idx), (s0, cnt, rr, idx, g, brute)
