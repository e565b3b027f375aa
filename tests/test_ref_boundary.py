"""CPU: the drop-in boundary against the reference's OWN header.

A translation unit includes /root/reference/src/ballet/ed25519/fd_ed25519.h
(real fd_sha512_t, FD_FN_CONST, uchar/ulong from fd_util_base.h) next to
include/fd_ed25519_hip.h, compiled with the oracle/Makefile machine -D flags
(config/machine/linux_gcc_icelake.mk's) and -Wall -Wextra -Werror:

- both declarations of each replaced symbol are in scope, so the compiler
  itself rejects any prototype mismatch ("conflicting types");
- each engine symbol is assigned to a function pointer of the reference's
  declared type;
- a caller shaped like fd_txn_verify (src/disco/verify/fd_verify_tile.h:93)
  calls fd_ed25519_verify_batch_single_msg( msg, msg_sz, sigs, pubs, shas,
  cnt ) and the program links against libfd_ed25519_hip.so and starts (no
  GPU call is made).

A negative control checks that the same compile fails when the engine's
prototype is perturbed, so a green test means the check bites.
Skipped where /root/reference is absent (the GPU box)."""
import os
import subprocess

import pytest

from firedancer_amd.build import LIB, build

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SRC = "/root/reference/src"
REF_HDR = os.path.join(REF_SRC, "ballet", "ed25519", "fd_ed25519.h")

# oracle/Makefile REF_COMMON + REF_AVXF defines (linux_gcc_icelake machine)
MACHINE = ["-std=c17", "-D_GNU_SOURCE", "-DFD_HAS_HOSTED=1", "-DFD_HAS_INT128=1", "-DFD_HAS_DOUBLE=1",
           "-DFD_HAS_ALLOCA=1", "-DFD_HAS_X86=1", "-march=icelake-server", "-DFD_HAS_SSE=1", "-DFD_HAS_AVX=1",
           "-DFD_HAS_AVX512=1", "-DFD_HAS_SHANI=1", "-DFD_HAS_GFNI=1", "-DFD_HAS_AESNI=1"]

CALLER = r"""
#include "ballet/ed25519/fd_ed25519.h"
#include "%(engine)s"
#include <stdio.h>

/* the reference's declared types (fd_ed25519.h:96-101, 124-130, 137-138) */
typedef int (*verify_fn_t)( uchar const *, ulong, uchar const *, uchar const *, fd_sha512_t * );
typedef int (*batch_fn_t)( uchar const *, ulong const, uchar const *, uchar const *, fd_sha512_t **,
                           uchar const );
typedef char const * (*strerror_fn_t)( int );

verify_fn_t   volatile ref_verify   = fd_ed25519_verify;
batch_fn_t    volatile ref_batch    = fd_ed25519_verify_batch_single_msg;
strerror_fn_t volatile ref_strerror = fd_ed25519_strerror;

/* fd_txn_verify's call, fd_verify_tile.h:93 */
int
txn_verify_shape( uchar const * msg, ulong msg_sz, uchar const * signatures, uchar const * pubkeys,
                  fd_sha512_t ** shas, uchar signature_cnt ) {
  return fd_ed25519_verify_batch_single_msg( msg, msg_sz, signatures, pubkeys, shas, signature_cnt );
}

int (* volatile caller)( uchar const *, ulong, uchar const *, uchar const *, fd_sha512_t **, uchar ) =
  txn_verify_shape;

int
main( void ) {
  /* host-only call (no GPU): the engine's strerror through the reference-typed pointer */
  printf( "%%s|%%s\n", ref_strerror( FD_ED25519_ERR_MSG ), fd_ed25519_strerror( FD_ED25519_ERR_PUBKEY ) );
  return (ref_verify && ref_batch && caller) ? 0 : 1;
}
"""

pytestmark = pytest.mark.skipif(not os.path.exists(REF_HDR), reason="/root/reference absent")


def _compile(tmp_path, engine_header, link=True):
    c = tmp_path / "caller.c"
    c.write_text(CALLER % {"engine": engine_header})
    exe = tmp_path / "caller"
    libdir = os.path.dirname(LIB)
    cmd = ["gcc", "-O2"] + MACHINE + ["-Wall", "-Wextra", "-Werror", "-I", REF_SRC,
                                     "-I", os.path.join(REPO, "include"), str(c)]
    if link:
        cmd += ["-L", libdir, "-lfd_ed25519_hip", "-Wl,-rpath-link,/opt/rocm/lib", "-Wl,-rpath," + libdir,
                "-o", str(exe)]
    else:
        cmd += ["-c", "-o", str(tmp_path / "caller.o")]
    return subprocess.run(cmd, capture_output=True, text=True), exe


def test_reference_header_binds_engine(tmp_path):
    build()
    r, exe = _compile(tmp_path, "fd_ed25519_hip.h")
    assert r.returncode == 0, r.stderr
    out = subprocess.check_output([str(exe)]).decode().strip()
    assert out == "bad message|bad public key"


def test_mismatched_prototype_is_rejected(tmp_path):
    """Negative control: the engine header with msg_sz narrowed to uint must
    not compile next to the reference declaration."""
    src = open(os.path.join(REPO, "include", "fd_ed25519_hip.h")).read()
    bad = src.replace("fd_ed25519_verify( uchar const                msg[], /* msg_sz */\n"
                      "                   ulong                      msg_sz,",
                      "fd_ed25519_verify( uchar const                msg[], /* msg_sz */\n"
                      "                   uint                       msg_sz,")
    assert bad != src
    h = tmp_path / "bad_engine.h"
    h.write_text(bad)
    r, _ = _compile(tmp_path, str(h), link=False)
    assert r.returncode != 0 and "conflicting types" in r.stderr, r.stderr


def _plug_flags(mode):
    """CPPFLAGS integration/with-hip.mk sets for FD_HIP_PLUG=mode (make -p of a
    Makefile that includes it)."""
    mk = os.path.join(REPO, "integration", "with-hip.mk")
    r = subprocess.run(["make", "-s", "-f", "-", f"FD_HIP_PLUG={mode}", "FD_HIP_ENGINE=" + REPO, "show"],
                       input=f"include {mk}\nshow:\n\t@echo $(CPPFLAGS)\n", capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return r.stdout.split()


def test_with_hip_mk_modes():
    """The build-side plug a maintainer drops into config/extra/ (INTEGRATION.md 1):
    selective by default (batch callers only), full on request, anything
    else refused."""
    sel, full = _plug_flags("selective"), _plug_flags("full")
    assert "-DFD_HAS_HIP=1" in sel and not any("DROPIN" in f for f in sel)
    assert "-DFD_HAS_HIP=1" in full and "-DFD_HAS_HIP_DROPIN=1" in full
    mk = os.path.join(REPO, "integration", "with-hip.mk")
    r = subprocess.run(["make", "-s", "-f", "-", "FD_HIP_PLUG=bogus", "show"],
                       input=f"include {mk}\nshow:\n\t@echo $(CPPFLAGS)\n", capture_output=True, text=True)
    assert r.returncode != 0 and "FD_HIP_PLUG" in r.stderr
    assert "-lfd_ed25519_hip" in open(mk).read()


PLUG_MAIN = r"""
#define _GNU_SOURCE
#include "ballet/ed25519/fd_ed25519.h"
#include <dlfcn.h>
#include <stdio.h>
#include <string.h>
int
main( void ) {
  /* the reference's own signer (patched fd_ed25519_user.c, CPU) still links */
  uchar prv[32], pub[32], sig[64], msg[3] = { 1, 2, 3 };
  fd_sha512_t sha[1];
  memset( prv, 7, 32 );
  fd_ed25519_public_from_private( pub, prv, sha );   /* init'd inside; no fd_log users linked */
  fd_ed25519_sign( sig, msg, 3, pub, prv, sha );
  /* ... while verify and strerror resolve to the engine's library */
  Dl_info a, b;
  if( !dladdr( (void *)fd_ed25519_verify, &a ) || !dladdr( (void *)fd_ed25519_strerror, &b ) ) return 2;
  printf( "%s|%s|%s|%02x%02x\n", strrchr( a.dli_fname, '/' ) + 1, strrchr( b.dli_fname, '/' ) + 1,
          fd_ed25519_strerror( FD_ED25519_ERR_SIG ), sig[0], sig[63] );
  return 0;
}
"""

REF_OBJS = ["ballet/ed25519/fd_curve25519.o", "ballet/ed25519/fd_curve25519_scalar.o", "ballet/ed25519/fd_f25519.o",
            "ballet/ed25519/avx512/fd_r43x6.o", "ballet/ed25519/avx512/fd_r43x6_ge.o", "ballet/sha512/fd_sha512.o",
            "ballet/sha512/fd_sha512_core_avx2.o"]


PLUG_SELECTIVE = r"""
#define _GNU_SOURCE
#include "ballet/ed25519/fd_ed25519.h"
#include "fd_replay_hip.h"
#include <dlfcn.h>
#include <stdio.h>
#include <string.h>
int
main( void ) {
  /* the reference's CPU verify stays in the program and answers the
     latency-bound callers ... */
  uchar prv[32], pub[32], sig[64], msg[3] = { 1, 2, 3 };
  fd_sha512_t sha[1];
  memset( prv, 7, 32 );
  fd_ed25519_public_from_private( pub, prv, sha );
  fd_ed25519_sign( sig, msg, 3, pub, prv, sha );
  int ok  = fd_ed25519_verify( msg, 3, sig, pub, sha );
  sig[5] ^= 1;
  int bad = fd_ed25519_verify( msg, 3, sig, pub, sha );
  /* ... while the batch callers' entry points come from the engine */
  Dl_info a, b;
  if( !dladdr( (void *)fd_ed25519_verify, &a ) || !dladdr( (void *)fd_replay_hip_txn_verify_host, &b ) ) return 2;
  char const * an = strrchr( a.dli_fname, '/' ), * bn = strrchr( b.dli_fname, '/' );
  printf( "%s|%s|%d|%d\n", an ? an+1 : a.dli_fname, bn ? bn+1 : b.dli_fname, ok, bad );
  return 0;
}
"""


def _patched_user_o(tmp_path, defs):
    src_dir = tmp_path / "src" / "ballet" / "ed25519"
    src_dir.mkdir(parents=True, exist_ok=True)
    user_c = src_dir / "fd_ed25519_user.c"
    user_c.write_text(open(os.path.join(REF_SRC, "ballet", "ed25519", "fd_ed25519_user.c")).read())
    subprocess.check_call(["patch", "-s", "-p1", "-d", str(tmp_path), "-i",
                           os.path.join(REPO, "integration", "fd_ed25519_user_hip.patch")])
    flags = ["-O2", "-ffunction-sections", "-fdata-sections"] + MACHINE + defs + ["-w", "-I", REF_SRC, "-I", str(src_dir)]
    # the patched file includes its siblings by relative path: compile it from the reference tree's view
    obj = tmp_path / "user.o"
    subprocess.check_call(["gcc"] + flags + ["-iquote", os.path.join(REF_SRC, "ballet", "ed25519"), "-c",
                                             str(user_c), "-o", str(obj)])
    return flags, obj


def _link_run(tmp_path, flags, obj, main_src, ref_o):
    main_c = tmp_path / "main.c"
    main_c.write_text(main_src)
    exe = tmp_path / "plug"
    libdir = os.path.dirname(LIB)
    r = subprocess.run(["gcc"] + flags + ["-I", os.path.join(REPO, "include"), str(main_c), str(obj)] +
                       [os.path.join(ref_o, o) for o in REF_OBJS] +
                       ["-Wl,--gc-sections",   # as oracle/Makefile: drop the unreferenced fd_log users
                        "-L", libdir, "-lfd_ed25519_hip", "-ldl", "-Wl,-rpath-link,/opt/rocm/lib",
                        "-Wl,-rpath," + libdir, "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return subprocess.check_output([str(exe)]).decode().strip().split("|")


def test_patched_reference_links_engine(tmp_path):
    """Full plug (FD_HIP_PLUG=full: -DFD_HAS_HIP=1 -DFD_HAS_HIP_DROPIN=1):
    integration/fd_ed25519_user_hip.patch applied to a temporary copy of the
    reference's fd_ed25519_user.c, compiled next to the reference's other
    verify-path objects (oracle/Makefile's build of the reference sources):
    the program links with no duplicate or missing symbol, the reference's
    CPU signer runs, and fd_ed25519_verify / strerror resolve to
    libfd_ed25519_hip.so."""
    ref_o = os.path.join(REPO, "oracle", "_ref", "avx512")
    if not all(os.path.exists(os.path.join(ref_o, o)) for o in REF_OBJS):
        pytest.skip("oracle/_ref reference objects not built")
    build()
    flags, obj = _patched_user_o(tmp_path, ["-DFD_HAS_HIP=1", "-DFD_HAS_HIP_DROPIN=1"])
    out = _link_run(tmp_path, flags, obj, PLUG_MAIN, ref_o)
    assert out[0] == "libfd_ed25519_hip.so" and out[1] == "libfd_ed25519_hip.so", out
    assert out[2] == "bad signature"


def test_selective_plug_keeps_cpu_verify(tmp_path):
    """Selective plug (the default, FD_HIP_PLUG=selective: -DFD_HAS_HIP=1
    alone): the same patched file keeps the reference's fd_ed25519_verify,
    which the program resolves to itself and which verifies on the CPU
    (SUCCESS, then ERR_MSG for a flipped signature bit, fd_ed25519.h:29-32),
    while the batch callers' engine entry points resolve to
    libfd_ed25519_hip.so; no GPU call is made."""
    ref_o = os.path.join(REPO, "oracle", "_ref", "avx512")
    if not all(os.path.exists(os.path.join(ref_o, o)) for o in REF_OBJS):
        pytest.skip("oracle/_ref reference objects not built")
    build()
    flags, obj = _patched_user_o(tmp_path, ["-DFD_HAS_HIP=1"])
    out = _link_run(tmp_path, flags, obj, PLUG_SELECTIVE, ref_o)
    assert out[0] == "plug" and out[1] == "libfd_ed25519_hip.so", out
    assert out[2] == "0" and int(out[3]) < 0, out
