#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Runs ONLY in the build container (it reads /root/reference and loads the
reference's own verify path compiled by oracle/Makefile into oracle/_ref/).
The fixtures are data: inputs plus the reference's verdicts.  Nothing in the
-m gpu tests, smoke() or bench.py reads /root/reference.

Sources (paths relative to /root/reference):
  src/ballet/ed25519/test_ed25519_wycheproof.c:22        133 Wycheproof vectors (+ ok flag)
  src/ballet/ed25519/test_ed25519_cctv.c:22              914 CCTV ed25519vectors (+ ok flag)
  src/ballet/ed25519/test_ed25519_signature_malleability_should_{fail,pass}.bin
                                                          196 + 200 (sig64||pub32), msg "Zcash"
  corpus/fuzz_ed25519_sigverify/*                         prv(32)||msg seeds (fuzz_ed25519_sigverify.c:25-53)
  src/ballet/ed25519/test_ed25519.c:1046-1050             sign KAT
  src/ballet/ed25519/test_ed25519.c:1266-1307             cctv batch (2/4 sigs, batch_single_msg)
plus seeded synthetic sets in the BASELINE config-2 mix (C2) signed and
verified by the reference build (both backends; their bitmaps must agree).

usage: python tests/golden/gen_golden.py   (after `make -C oracle all`)
"""
import ctypes
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("FD_REFERENCE", "/root/reference")
ED = os.path.join(REF, "src/ballet/ed25519")

sys.path.insert(0, os.path.join(REPO, "tests"))
from fdgen import c2_mutate, L_INT, P_INT  # noqa: E402  (repo-owned mutation model)


class RefLib:
    """ctypes binding to one reference build (oracle/_ref/libfdref_*.so)."""

    def __init__(self, path):
        self.lib = ctypes.CDLL(path)
        self.lib.fd_ed25519_verify.restype = ctypes.c_int
        self.lib.fd_ed25519_verify.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p,
                                               ctypes.c_char_p, ctypes.c_void_p]
        self.lib.fd_ed25519_verify_batch_single_msg.restype = ctypes.c_int
        self.lib.fd_ed25519_verify_batch_single_msg.argtypes = [
            ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p,
            ctypes.POINTER(ctypes.c_void_p), ctypes.c_ubyte]
        self.lib.fd_ed25519_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_ulong,
                                             ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
        self.lib.fd_ed25519_public_from_private.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
        self.lib.fd_sha512_init.restype = ctypes.c_void_p
        self.lib.fd_sha512_init.argtypes = [ctypes.c_void_p]
        # 16 sha objects: footprint 256, align 128 (fd_sha512.h:56-77)
        self._buf = ctypes.create_string_buffer(256 * 17)
        base = (ctypes.addressof(self._buf) + 127) & ~127
        self.shas = (ctypes.c_void_p * 16)(*[base + 256 * i for i in range(16)])
        for i in range(16):
            self.lib.fd_sha512_init(self.shas[i])

    def verify(self, msg, sig, pub):
        return self.lib.fd_ed25519_verify(msg, len(msg), sig, pub, self.shas[0])

    def batch(self, msg, sigs, pubs, n):
        return self.lib.fd_ed25519_verify_batch_single_msg(msg, len(msg), sigs, pubs, self.shas, n)

    def pub_from_prv(self, prv):
        out = ctypes.create_string_buffer(32)
        self.lib.fd_ed25519_public_from_private(out, prv, self.shas[0])
        return out.raw

    def sign(self, msg, pub, prv):
        out = ctypes.create_string_buffer(64)
        self.lib.fd_ed25519_sign(out, msg, len(msg), pub, prv, self.shas[0])
        return out.raw


def _cstr(s):
    """Decode a C string literal body ("\\x12\\x34..." or plain chars)."""
    out = bytearray()
    i = 0
    while i < len(s):
        if s[i] == "\\":
            if s[i + 1] == "x":
                out.append(int(s[i + 2:i + 4], 16)); i += 4; continue
            esc = {"n": 10, "t": 9, "0": 0, "\\": 92, '"': 34}
            out.append(esc[s[i + 1]]); i += 2; continue
        out.append(ord(s[i])); i += 1
    return bytes(out)


def parse_vector_file(path):
    txt = open(path).read()
    recs = []
    for m in re.finditer(r"\{\s*\.tc_id\s*=\s*(\d+),\s*\.comment\s*=\s*\"(.*?)\",\s*"
                         r"\.msg\s*=\s*\(uchar const \*\)\"(.*?)\",\s*\.msg_sz\s*=\s*(\d+)UL,\s*"
                         r"\.sig\s*=\s*\"(.*?)\",\s*\.pub\s*=\s*\"(.*?)\",\s*\.ok\s*=\s*(\d+)\s*\}", txt, re.S):
        tc, comment, msg, msg_sz, sig, pub, ok = m.groups()
        msg = _cstr(msg)
        assert len(msg) == int(msg_sz), (path, tc)
        sig, pub = _cstr(sig), _cstr(pub)
        assert len(sig) == 64 and len(pub) == 32
        recs.append(dict(tc_id=int(tc), comment=comment, msg=msg.hex(), sig=sig.hex(), pub=pub.hex(), ok=int(ok)))
    return recs


def add_ref_verdicts(recs, avx, ref):
    for r in recs:
        msg, sig, pub = bytes.fromhex(r["msg"]), bytes.fromhex(r["sig"]), bytes.fromhex(r["pub"])
        r["code_avx512"] = avx.verify(msg, sig, pub)
        r["code_ref"] = ref.verify(msg, sig, pub)
        assert (r["code_avx512"] == 0) == (r["code_ref"] == 0), r
        if "ok" in r:
            assert (r["code_avx512"] == 0) == bool(r["ok"]), r


def main():
    avx = RefLib(os.path.join(REPO, "oracle/_ref/libfdref_avx512.so"))
    ref = RefLib(os.path.join(REPO, "oracle/_ref/libfdref_ref.so"))
    golden = {}

    # --- Wycheproof / CCTV -------------------------------------------------
    wy = parse_vector_file(os.path.join(ED, "test_ed25519_wycheproof.c"))
    cc = parse_vector_file(os.path.join(ED, "test_ed25519_cctv.c"))
    assert len(wy) == 145 or len(wy) >= 133, len(wy)
    assert len(cc) == 914, len(cc)
    add_ref_verdicts(wy, avx, ref)
    add_ref_verdicts(cc, avx, ref)
    golden["wycheproof"] = wy
    golden["cctv"] = cc

    # --- malleability --------------------------------------------------------
    mal = []
    for name, ok in (("should_fail", 0), ("should_pass", 1)):
        raw = open(os.path.join(ED, f"test_ed25519_signature_malleability_{name}.bin"), "rb").read()
        assert len(raw) % 96 == 0
        for i in range(len(raw) // 96):
            rec = raw[96 * i:96 * (i + 1)]
            mal.append(dict(tc_id=i, comment=name, msg=b"Zcash".hex(), sig=rec[:64].hex(), pub=rec[64:].hex(), ok=ok))
    add_ref_verdicts(mal, avx, ref)
    golden["malleability"] = mal

    # --- fuzz corpus seeds: prv(32)||msg -> sign -> verify must pass ---------
    corp = []
    cdir = os.path.join(REF, "corpus/fuzz_ed25519_sigverify")
    for fn in sorted(os.listdir(cdir)):
        raw = open(os.path.join(cdir, fn), "rb").read()
        if len(raw) < 32:
            continue
        prv, msg = raw[:32], raw[32:]
        pub = avx.pub_from_prv(prv)
        sig = avx.sign(msg, pub, prv)
        assert ref.sign(msg, ref.pub_from_prv(prv), prv) == sig
        corp.append(dict(tc_id=len(corp), comment=fn, prv=prv.hex(), msg=msg.hex(), sig=sig.hex(), pub=pub.hex(), ok=1))
    add_ref_verdicts(corp, avx, ref)
    golden["corpus"] = corp

    # --- sign KAT (test_ed25519.c:1046-1050) ---------------------------------
    prv = bytes.fromhex("57835dc6a20e4efd70e90882dbd832b577dbc469960284e0ee718fb526d2ec84")
    exp = bytes.fromhex("d65759870ce42b34fd955871f0371ce1c9a976edbe98417b84541bb4c68b65a0"
                        "673799895c61d530624ffbf92c047d47d4eb4cd1bac2ecee1365faebb53a6303")
    pub = avx.pub_from_prv(prv)
    assert avx.sign(b"", pub, prv) == exp
    golden["sign_kat"] = [dict(prv=prv.hex(), pub=pub.hex(), msg="", sig=exp.hex())]

    # --- cctv batch: batch_single_msg with the cctv case spliced at j=1 ------
    rng = np.random.default_rng(0x5eed0003)
    msg7 = bytes.fromhex(cc[7]["msg"])
    pubs, sigs = [], []
    for j in range(16):
        p = rng.bytes(32)
        pk = avx.pub_from_prv(p)
        pubs.append(pk); sigs.append(avx.sign(msg7, pk, p))
    batch = []
    for r in cc:
        if bytes.fromhex(r["msg"]) != msg7:
            continue
        S = list(sigs); P = list(pubs)
        S[1] = bytes.fromhex(r["sig"]); P[1] = bytes.fromhex(r["pub"])
        for n in (2, 4):
            sb, pb = b"".join(S[:n]), b"".join(P[:n])
            ca, cr = avx.batch(msg7, sb, pb, n), ref.batch(msg7, sb, pb, n)
            assert (ca == 0) == bool(r["ok"]) and (cr == 0) == (ca == 0)
            batch.append(dict(tc_id=r["tc_id"], n=n, msg=msg7.hex(), sigs=sb.hex(), pubs=pb.hex(),
                              code_avx512=ca, code_ref=cr, ok=r["ok"]))
    # batch size edge cases: 0 and 17 -> ERR_SIG (fd_ed25519_user.c:238-241)
    sb, pb = b"".join(sigs) + sigs[0], b"".join(pubs) + pubs[0]
    for n in (0, 16, 17):
        batch.append(dict(tc_id=-1, n=n, msg=msg7.hex(), sigs=sb[:64 * max(n, 1)].hex(), pubs=pb[:32 * max(n, 1)].hex(),
                          code_avx512=avx.batch(msg7, sb, pb, n), code_ref=ref.batch(msg7, sb, pb, n), ok=int(n == 16)))
    golden["cctv_batch"] = batch

    with open(os.path.join(HERE, "kat_vectors.json"), "w") as f:
        json.dump(golden, f, indent=0, separators=(",", ":"))

    # --- seeded C2-mix synthetic set (binary fixture, no pickle) -------------
    n = 4096
    rng = np.random.default_rng(0x5eed0002)
    prvs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    msz = rng.integers(0, 300, size=n).astype(np.uint32)
    msz[: n // 2] = 64                                     # half at the C1 message size
    moff = np.zeros(n, np.uint32); moff[1:] = np.cumsum(msz)[:-1]
    pool = rng.integers(0, 256, size=int(msz.sum()) + 1, dtype=np.uint8)
    sigs = np.zeros((n, 64), np.uint8); pubs = np.zeros((n, 32), np.uint8)
    for i in range(n):
        pk = avx.pub_from_prv(prvs[i].tobytes())
        m = pool[moff[i]:moff[i] + msz[i]].tobytes()
        pubs[i] = np.frombuffer(pk, np.uint8)
        sigs[i] = np.frombuffer(avx.sign(m, pk, prvs[i].tobytes()), np.uint8)
    kinds = c2_mutate(sigs, pubs, np.random.default_rng(0x5eed0004))
    ca = np.zeros(n, np.int8); cr = np.zeros(n, np.int8)
    for i in range(n):
        m = pool[moff[i]:moff[i] + msz[i]].tobytes()
        ca[i] = avx.verify(m, sigs[i].tobytes(), pubs[i].tobytes())
        cr[i] = ref.verify(m, sigs[i].tobytes(), pubs[i].tobytes())
    assert np.array_equal(ca == 0, cr == 0)
    np.savez_compressed(os.path.join(HERE, "c2_mix_4096.npz"), sigs=sigs, pubs=pubs, msg_off=moff, msg_sz=msz,
                        pool=pool, kinds=kinds, code_avx512=ca, code_ref=cr)
    print("wycheproof", len(wy), "cctv", len(cc), "malleability", len(mal), "corpus", len(corp),
          "cctv_batch", len(batch), "c2 accept", float((ca == 0).mean()))
    print("c2 codes avx512", {int(k): int(v) for k, v in zip(*np.unique(ca, return_counts=True))},
          "ref", {int(k): int(v) for k, v in zip(*np.unique(cr, return_counts=True))})


if __name__ == "__main__":
    main()
