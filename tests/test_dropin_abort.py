"""CPU: the drop-in entry points abort loudly on a message the engine cannot
address (msg_sz beyond its 32-bit offsets), in a child process, before any
GPU call -- never a silent verdict over a truncated prefix (SURVEY.md 8(b)
"Errors"; fd_ed25519.h:96-101 takes a ulong msg_sz)."""
import subprocess
import sys

import pytest

from firedancer_amd.build import LIB, build

CHILD = r"""
import ctypes, sys
L = ctypes.CDLL(sys.argv[1])
fn = sys.argv[2]
c = ctypes
buf = c.create_string_buffer(64)
if fn == "verify":
    L.fd_ed25519_verify.argtypes = [c.c_char_p, c.c_ulong, c.c_char_p, c.c_char_p, c.c_void_p]
    L.fd_ed25519_verify(b"x", int(sys.argv[3]), buf.raw, buf.raw[:32], None)
else:
    L.fd_ed25519_verify_batch_single_msg.argtypes = [c.c_char_p, c.c_ulong, c.c_char_p, c.c_char_p, c.c_void_p,
                                                     c.c_ubyte]
    L.fd_ed25519_verify_batch_single_msg(b"x", int(sys.argv[3]), buf.raw, buf.raw[:32], None, 1)
print("returned")
"""


@pytest.mark.parametrize("fn", ["verify", "batch"])
@pytest.mark.parametrize("msg_sz", [1 << 32, (1 << 32) - 1, (1 << 64) - 1])
def test_oversize_message_aborts(fn, msg_sz):
    build()
    r = subprocess.run([sys.executable, "-c", CHILD, LIB, fn, str(msg_sz)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == -6, (r.returncode, r.stdout, r.stderr[-2000:])      # SIGABRT
    assert "returned" not in r.stdout
    assert "exceeds the engine's 32-bit message limit" in r.stderr


def test_batch_size_checked_before_size():
    """batch_sz 0 / >16 is ERR_SIG (fd_ed25519_user.c:238-241) whatever msg_sz
    is: that check precedes the size check, as in the reference, and needs no
    GPU."""
    build()
    code = (CHILD.split("if fn ==")[0] +
            "L.fd_ed25519_verify_batch_single_msg.argtypes = [c.c_char_p, c.c_ulong, c.c_char_p, c.c_char_p, "
            "c.c_void_p, c.c_ubyte]\n"
            "print(L.fd_ed25519_verify_batch_single_msg(b'x', 1 << 40, buf.raw, buf.raw[:32], None, 0),"
            " L.fd_ed25519_verify_batch_single_msg(b'x', 1 << 40, buf.raw, buf.raw[:32], None, 17))\n")
    r = subprocess.run([sys.executable, "-c", code, LIB, "batch", "0"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split() == ["-1", "-1"]
