"""Static ISA histogram of one engine kernel, per loop (backward-branch body).

usage: python tools/isa_hist.py [lib] [kernel substring]
Prints each loop body (> 50 instructions) with its opcode counts: the window
and doubling loops of k_verify_dsm are where the dynamic instruction count
lives, so A/B builds are compared here before they go to the GPU."""
import collections
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from firedancer_amd.kernel_hash import _bundles, _elf_symbols  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def kernel_insts(lib, kernel):
    blob = open(lib, "rb").read()
    for ident, co in _bundles(blob):
        if "gfx950" not in ident:
            continue
        syms, _ = _elf_symbols(co)
        hit = [s for s in syms if kernel in s[0] and not s[0].endswith(".kd") and s[2]]
        if not hit:
            continue
        name, start, size, _ = hit[0]
        path = "/tmp/_isa_hist.co"
        with open(path, "wb") as f:
            f.write(co)
        out = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", path], capture_output=True, text=True).stdout
        insts = []
        for line in out.split("\n"):
            m = re.match(r"\s+(\w[\w.]*)\s*(.*?)\s*//\s*([0-9A-F]+):.*?(?:<[^+>]+\+0x([0-9a-f]+)>)?$", line.rstrip())
            if m:
                a = int(m.group(3), 16)
                if start <= a < start + size:
                    tgt = start + int(m.group(4), 16) if m.group(4) else None
                    insts.append((a, m.group(1), tgt))
        return name, insts
    raise SystemExit(f"{kernel} not found in {lib}")


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "firedancer_amd",
                                                              "libfd_ed25519_hip.so")
    kernel = sys.argv[2] if len(sys.argv) > 2 else "k_verify_dsm"
    name, insts = kernel_insts(lib, kernel)
    tot = collections.Counter(op for _, op, _ in insts)
    print(name, "static", len(insts), "valu", sum(v for k, v in tot.items() if k.startswith("v_")))
    seen = set()
    for a, op, tgt in insts:
        if (op.startswith("s_cbranch") or op == "s_branch") and tgt is not None and tgt <= a:
            body = [x for x in insts if tgt <= x[0] <= a]
            if len(body) > 50 and (tgt, a) not in seen:
                seen.add((tgt, a))
                c = collections.Counter(x[1] for x in body)
                print(f"loop {tgt:#x}-{a:#x}: {len(body)} insts, valu {sum(v for k, v in c.items() if k.startswith('v_'))}")
                print("   ", ", ".join(f"{k} {v}" for k, v in c.most_common(16)))


if __name__ == "__main__":
    main()
