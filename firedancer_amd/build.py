"""Build the gfx950 engine in-tree: firedancer_amd/libfd_ed25519_hip.so.

One hipcc invocation (--offload-arch=gfx950) producing a C-ABI shared
library.  hipcc cross-compiles without a GPU, so this runs in the build
container too.
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libfd_ed25519_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["fd_ed25519_hip.hip", "fd_ed25519_dev.h", "fd_hip_order.h", "fd_txn_hip.hip", "fd_txn_hip_int.h", "fd_sha512_hip.hip",
           "fd_verify_svc.hip"]
UNITS = ["fd_ed25519_hip.hip", "fd_txn_hip.hip", "fd_sha512_hip.hip", "fd_verify_svc.hip"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def variant_path(name):
    return LIB if not name else os.path.join(PKG, f"libfd_ed25519_hip_{name}.so")


def build(force=False, verbose=False, variant=None, defines=()):
    """Build the library (or an experimental variant with extra -D defines,
    loaded when FD_ED25519_HIP_LIB names it)."""
    lib_path = variant_path(variant)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(PKG, "..", "include", h) for h in ("fd_ed25519_hip.h", "fd_verify_hip.h", "fd_replay_hip.h", "fd_sha512_hip.h", "fd_verify_svc.h")]
    if force or _stale(lib_path, deps):
        extra = os.environ.get("FD_HIPCC_EXTRA", "").split() if variant else []   # variants only: A/B flags
        cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17"] + extra + \
              [f"-D{d}" for d in defines] + ["-o", lib_path + ".tmp"] + [os.path.join(CSRC, u) for u in UNITS]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
        os.replace(lib_path + ".tmp", lib_path)
    return lib_path


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    if args:   # python build.py <variant> DEF=1 ...
        print(build(force="--force" in sys.argv, verbose=True, variant=args[0], defines=args[1:]))
    else:
        print(build(force="--force" in sys.argv, verbose=True))
