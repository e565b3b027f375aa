"""Build the gfx950 engine in-tree: firedancer_amd/libfd_ed25519_hip.so.

Steps: regenerate csrc/fe25519_asm.h from csrc/gen_fe_asm.py, then one hipcc
invocation (--offload-arch=gfx950) producing a C-ABI shared library.  hipcc
cross-compiles without a GPU, so this runs in the build container too.
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libfd_ed25519_hip.so")
SCRATCH_BASE = os.environ.get("FE_SCRATCH_BASE", "124")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["fd_ed25519_hip.hip", "fd_ed25519_dev.h", "gen_fe_asm.py"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    asm_h = os.path.join(CSRC, "fe25519_asm.h")
    gen = os.path.join(CSRC, "gen_fe_asm.py")
    env = dict(os.environ, FE_SCRATCH_BASE=SCRATCH_BASE)
    if force or _stale(asm_h, [gen]) or f"FE_ASM_SCRATCH_BASE {SCRATCH_BASE}\n" not in open(asm_h).read():
        subprocess.check_call([sys.executable, gen, asm_h], env=env)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [asm_h, os.path.join(PKG, "..", "include", "fd_ed25519_hip.h")]
    if force or _stale(LIB, deps):
        cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
               "-o", LIB + ".tmp", os.path.join(CSRC, "fd_ed25519_hip.hip")]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
        os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
