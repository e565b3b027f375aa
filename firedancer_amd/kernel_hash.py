"""Identify the machine code of a kernel in the engine library (no tools).

The gfx950 code objects live in the library's .hip_fatbin section as clang
offload bundles ("__CLANG_OFFLOAD_BUNDLE__", one per translation unit).  Each
bundle entry for amdgcn-amd-amdhsa--gfx950 is an ELF whose symbol table gives
every kernel's address and size in .text.  kernel_hashes() returns a short
sha256 of those bytes per kernel name, so a committed profile summary can
record which build it measured and bench.py can tell when the library it
loaded differs (the summary's counters then describe other code)."""
import hashlib
import os
import struct

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _bundles(blob):
    at = 0
    while True:
        i = blob.find(MAGIC, at)
        if i < 0:
            return
        n, = struct.unpack_from("<Q", blob, i + 24)
        p = i + 32
        for _ in range(n):
            off, size, idlen = struct.unpack_from("<QQQ", blob, p)
            ident = blob[p + 24:p + 24 + idlen].decode(errors="replace")
            p += 24 + idlen
            yield ident, blob[i + off:i + off + size]
        at = i + len(MAGIC)


def _elf_symbols(elf):
    """(name, value, size, section index) of every symbol of a 64-bit ELF."""
    if elf[:4] != b"\x7fELF":
        return [], []
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + k * shentsize) for k in range(shnum)]
    out = []
    for name, typ, flags, addr, off, size, link, info, align, entsize in secs:
        if typ != 2:                                  # SHT_SYMTAB
            continue
        strtab = secs[link]
        for k in range(size // 24):
            st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", elf, off + 24 * k)
            e = elf.index(b"\0", strtab[4] + st_name)
            out.append((elf[strtab[4] + st_name:e].decode(errors="replace"), st_value, st_size, st_shndx))
    return out, secs


def kernel_hashes(lib_path, names=("k_verify_dsm", "k_verify_prep")):
    """{kernel name: 16-hex-digit sha256 of its gfx950 machine code}."""
    with open(lib_path, "rb") as f:
        blob = f.read()
    found = {}
    for ident, co in _bundles(blob):
        if "gfx950" not in ident:
            continue
        syms, secs = _elf_symbols(co)
        for sname, value, size, shndx in syms:
            for k in names:
                # C++-mangled kernel symbol: _Z<len><name>...; "name<N>" names the
                # int-template instance _Z<len><name>ILi<N>E...; skip the .kd descriptor
                if "<" in k:
                    base, arg = k[:-1].split("<")
                    pat = f"{len(base)}{base}ILi{arg}E"
                else:
                    pat = f"{len(k)}{k}"
                if pat in sname and not sname.endswith(".kd") and size and 0 < shndx < len(secs):
                    sec = secs[shndx]
                    start = sec[4] + (value - sec[3])
                    found[k] = hashlib.sha256(co[start:start + size]).hexdigest()[:16]
    return found


def engine_kernel_hashes(names=("k_verify_dsm", "k_verify_prep")):
    from .ed25519 import LIB
    path = os.environ.get("FD_ED25519_HIP_LIB") or LIB
    return kernel_hashes(path, names)


if __name__ == "__main__":
    import sys
    print(kernel_hashes(sys.argv[1] if len(sys.argv) > 1 else
                        os.path.join(os.path.dirname(os.path.abspath(__file__)), "libfd_ed25519_hip.so")))
